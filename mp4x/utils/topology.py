"""Local GPU topology: which device pairs are one xGMI hop apart (native probe csrc/runtime/topo.hip).

mp4x's device schedules are laid out for the MI355X node: 8 GPUs, a full mesh of point-to-point
xGMI links (7 per GPU), peer HBM readable by kernels through IPC / VMM mappings.  The reference
has no topology notion (slaves on 1 GbE, /root/reference/README.md:300); here the probe

* is recorded by ``bench.py`` next to every result (evidence that a multi-GPU run crossed xGMI
  and not PCIe); the autotuners decide schedules from measurements either way, so a PCIe-only
  box still runs, just without the claim.

:func:`summarize` is a pure function over the probe's matrices (unit-tested on CPU).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence

LINK_NAMES = {0: "hypertransport", 1: "qpi", 2: "pcie", 3: "infiniband", 4: "xgmi"}
XGMI = 4
_MAX_DEVICES = 64

_sig_done = False


def _lib():
    global _sig_done
    from ..ops import native
    lib = native.hip()
    if not _sig_done:
        ip = ctypes.POINTER(ctypes.c_int)
        native.register_signatures({"mp4x_topology": (ctypes.c_int, [ctypes.c_int, ip, ip, ip, ip, ip])})
        _sig_done = True
    return lib


def probe() -> Optional[Dict[str, List[List[int]]]]:
    """Raw n x n matrices of the visible devices (``link``, ``hops``, ``access``, ``perf_rank``,
    ``atomics``), or None without a GPU / native library."""
    try:
        import torch
        if not torch.cuda.is_available():
            return None
        lib = _lib()
    except Exception:   # noqa: BLE001 — CPU container, library not built
        return None
    cap = _MAX_DEVICES
    arrs = [(ctypes.c_int * (cap * cap))() for _ in range(5)]
    n = lib.mp4x_topology(cap, *arrs)
    if n <= 0:
        return None
    names = ("link", "hops", "access", "perf_rank", "atomics")
    return {k: [[a[i * n + j] for j in range(n)] for i in range(n)] for k, a in zip(names, arrs)}


def summarize(m: Dict[str, List[List[int]]], devices: Optional[Sequence[int]] = None) -> Dict:
    """Summary of the pairs among ``devices`` (default: every probed device): link-type counts,
    max hop count, whether every pair is a peer-accessible single xGMI hop (``xgmi_mesh``)."""
    n = len(m["link"])
    devs = list(range(n)) if devices is None else [d for d in devices if 0 <= d < n]
    devs = list(dict.fromkeys(devs))
    kinds: Dict[str, int] = {}
    max_hops = 0
    mesh = True
    no_access = []
    for a in devs:
        for b in devs:
            if a == b:
                continue
            lt = m["link"][a][b]
            kinds[LINK_NAMES.get(lt, "unknown")] = kinds.get(LINK_NAMES.get(lt, "unknown"), 0) + 1
            max_hops = max(max_hops, m["hops"][a][b])
            if not m["access"][a][b]:
                no_access.append((a, b))
            if lt != XGMI or m["hops"][a][b] != 1 or not m["access"][a][b]:
                mesh = False
    return {"devices": len(devs), "pairs": kinds, "max_hops": max_hops,
            "xgmi_mesh": mesh if len(devs) > 1 else None, "no_peer_access": no_access[:8]}


def local_summary(devices: Optional[Sequence[int]] = None) -> Optional[Dict]:
    """:func:`summarize` of :func:`probe` (None without a GPU)."""
    m = probe()
    return None if m is None else summarize(m, devices)
