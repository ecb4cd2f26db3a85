"""Rank-count-aware size tiers of the staged IPC allreduce, and the topology-keyed tune store
(VERDICT r5 Next #4).

**Per-link byte model** (DESIGN.md §6).  On a full xGMI mesh every rank has a link of its own to
each peer, so a schedule's time is its cross-rank barrier round trips plus the bytes the busiest
link carries:

* one-shot: every rank reads all S bytes of every peer — S over each link, and ONE barrier
  (slotted, no end barrier);
* two-shot: direct reduce-scatter + direct all-gather — 2S/p over each link, and TWO barriers.

    T1(S) = b + S / L          T2(S) = 2b + 2S / (p L)

so the one-shot wins below S* = b L / (1 - 2/p).  At p = 2 the two cost the same bytes and the
one-shot saves a barrier at every size: two ranks take it up to the slot that holds a staged call
(4 MiB).  b (one cross-GPU flag round trip, µs) and L (achieved GB/s per link and direction) are
model constants, ``MP4X_TIER_BARRIER_US`` (2.5) and ``MP4X_TIER_LINK_GBPS`` (64: about 85 % of an
MI355X xGMI link's one-direction rate); S* is rounded to the nearest power of two and clamped to
[64 KiB, slot].  The defaults this gives: p = 2 → 4 MiB (the slot), 3 → 512 KiB, 4..8 → 256 KiB.
Autotune replaces the model by measurement for every size class it visits, and those pins persist
(below).

**Tune store.**  The tier sweep of ``bench.py`` autotunes every size class from 4 KiB to 64 MiB
on the job's real links; with ``MP4X_TUNE_AUTO=1`` (bench.py sets it) the pinned table is written
to ``MP4X_TUNE_DIR`` (``~/.cache/mp4x/tune``) under a file named after the job's topology key —
rank count, device name, backend, node count and the xGMI pair map of the ranks' devices
(``mp4x.utils.topology``) — and every later communicator with the same key loads it at creation
(rank 0 reads, every rank pins rank 0's copy).  A table under another key is never read; a table
whose recorded topology differs from the job's is refused (``load_tuning``).
Reference: the per-collective alpha-beta cost model of /root/reference/README.md:286-294.
"""
from __future__ import annotations

import hashlib
import json
import math
import os
from typing import Optional

MIN_ONESHOT = 64 << 10


def model_constants():
    """(barrier µs, link GB/s) of the per-link model."""
    return (float(os.environ.get("MP4X_TIER_BARRIER_US", 2.5)), float(os.environ.get("MP4X_TIER_LINK_GBPS", 64.0)))


def oneshot_crossover(p: int, barrier_us: Optional[float] = None, link_gbps: Optional[float] = None) -> float:
    """S* in bytes (inf at p <= 2: the one-shot never loses there)."""
    b, L = model_constants()
    b = b if barrier_us is None else barrier_us
    L = L if link_gbps is None else link_gbps
    if p <= 2:
        return math.inf
    return b * 1e-6 * L * 1e9 / (1.0 - 2.0 / p)


def oneshot_max(p: int, slot_bytes: int, barrier_us: Optional[float] = None,
                link_gbps: Optional[float] = None) -> int:
    """Largest staged allreduce that runs the one-shot at ``p`` ranks (the model's S*, rounded to
    the nearest power of two, within [64 KiB, slot])."""
    s = oneshot_crossover(p, barrier_us, link_gbps)
    if slot_bytes <= 0:
        slot_bytes = 256 << 10
    if math.isinf(s):
        return int(slot_bytes)
    r = 1 << int(round(math.log2(max(s, 1.0))))
    return int(min(max(r, MIN_ONESHOT), slot_bytes))


def model_times_us(p: int, nbytes: int, barrier_us: Optional[float] = None, link_gbps: Optional[float] = None):
    """(one-shot, two-shot) model times in µs of an ``nbytes`` staged allreduce (for records)."""
    b, L = model_constants()
    b = b if barrier_us is None else barrier_us
    L = (L if link_gbps is None else link_gbps) * 1e3          # bytes per µs
    return b + nbytes / L, 2 * b + 2 * nbytes / (p * L)


# ---------------------------------------------------------------- topology-keyed tune store
def auto_enabled() -> bool:
    return os.environ.get("MP4X_TUNE_AUTO", "0") == "1"


def tune_dir() -> str:
    return os.environ.get("MP4X_TUNE_DIR") or os.path.join(os.path.expanduser("~"), ".cache", "mp4x", "tune")


def topology_key(topology: dict) -> str:
    """Stable short key of a topology record (the file name of its tune table)."""
    blob = json.dumps(topology, sort_keys=True, separators=(",", ":"), default=str)
    return hashlib.sha1(blob.encode()).hexdigest()[:16]


def tune_path(topology: dict) -> str:
    return os.path.join(tune_dir(), f"tune-p{topology.get('p', 'x')}-{topology_key(topology)}.json")


def xgmi_map(p: int, device_index: Optional[int]):
    """The xGMI pair map of the ranks' devices (one process per GPU: devices 0..p-1 of the node;
    ranks sharing one GPU: that device alone), or None without a GPU / native library."""
    try:
        import torch
        from ..utils import topology as topo
        if not torch.cuda.is_available():
            return None
        devs = list(range(p)) if torch.cuda.device_count() >= p else [int(device_index or 0)]
        m = topo.probe()
        if m is None:
            return None
        s = topo.summarize(m, devs)
        return {"devices": s["devices"], "pairs": s["pairs"], "max_hops": s["max_hops"], "xgmi_mesh": s["xgmi_mesh"]}
    except Exception:   # noqa: BLE001 — the key just carries no link map then
        return None
