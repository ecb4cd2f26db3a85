"""Co-residency grid caps of the IPC per-block-barrier kernels (csrc/runtime/ipc*.hip).

Block b of every rank meets block b of its peers at each barrier, so every rank's block b must be
resident at the same time.  With one process per MI355X that always holds (grid <= 256 blocks,
one GPU each).  When several ranks share ONE GPU (the single-GPU rehearsals and tests), all of
their blocks share that GPU's resident-block budget, and a grid too large for it stalls at the
first barrier until the spin bound expires.

The budget is derived per launched kernel instantiation (family, dtype, kernel op, rank count),
not guessed per library:

* the occupancy API (``hipOccupancyMaxActiveBlocksPerMultiprocessor``, via the
  ``mp4x_ipc_occupancy_*`` entry points), and
* the compiler's own resource usage of that kernel (``-Rpass-analysis=kernel-resource-usage``,
  saved by tools/build_native.py into ``mp4x/_native/ipc_kernel_resources.json``), turned into
  blocks per CU with the CDNA4 residency rules (512 VGPRs per SIMD lane in granules of 8, 800
  SGPRs per SIMD at ``ceil(sgpr / 16) * 16 + 16`` per wave, 160 KiB LDS per CU, 8 waves per SIMD).
  The API alone over-reports by one block per CU for SGPR-heavy kernels on ROCm 7.2
  (cdna_hip_programming.md §1), so the smaller of the two answers is used.

The shared-GPU cap is ``CUs * bpc // (2 * share)``: the ranks sharing a GPU get half of its
resident capacity between them — the other half absorbs the ranks' own non-IPC kernels (quantise,
copies, torch) and dispatch imbalance across the 8 XCDs.  With the full capacity (fp8 two-shot at
8 ranks: 2 blocks per CU, 64 blocks per rank) the ranks stalled at the start barrier; with half
(32 per rank) config 5 runs exact (profiles/r3/configs_s2/README.md).
"""
from __future__ import annotations

import json
import os
import re
from typing import Dict, Optional, Tuple

THREADS = 512              # kIpcThreads
SIMDS_PER_CU = 4
MAX_WAVES_PER_SIMD = 8
VGPRS_PER_SIMD_LANE = 512  # unified arch + acc VGPR file (wave64)
SGPRS_PER_SIMD = 800
LDS_PER_CU = 160 * 1024
MAX_BLOCKS = 256           # kIpcMaxBlocks

# kernel-op template value of a (dtype, op) pair, mirroring ipc_common.hpp with_op():
# hot pairs keep their op, every other pair runs the runtime-op kernel (-1)
_HOT_SUM = {"F64", "F32", "I64", "I32", "BF16", "F16"}
_HOT_MINMAX = {"F32", "BF16", "F16"}
_FAMILY_KERNEL = {"oneshot": "k_ipc_oneshot", "twoshot": "k_ipc_twoshot", "push": "k_ipc_twoshot_push",
                  "rs": "k_ipc_reduce_range", "gather": "k_ipc_gather", "plan": "k_ipc_copy_plan",
                  "fp8": "k_ipc_fp8_twoshot", "fp8n": "k_ipc_fp8_twoshot_narrow"}


def kernel_op(dtype_name: str, op_code: int) -> int:
    """Template op of the kernel a (dtype, op) call launches (SUM = 0, MAX = 1, MIN = 2)."""
    if op_code == 0 and dtype_name in _HOT_SUM:
        return 0
    if op_code in (1, 2) and dtype_name in _HOT_MINMAX:
        return op_code
    return -1


def blocks_per_cu(res: Dict[str, int], threads: int = THREADS) -> int:
    """Resident blocks of ``threads`` per CU for a kernel with resources ``res`` (sgpr, vgpr,
    agpr, lds, occ = the compiler's waves/SIMD)."""
    waves_block = max(1, -(-threads // 64))
    vg = max(1, int(res.get("vgpr", 0)) + int(res.get("agpr", 0)))
    vg_alloc = -(-vg // 8) * 8
    w_v = VGPRS_PER_SIMD_LANE // vg_alloc
    sg_alloc = -(-max(1, int(res.get("sgpr", 0))) // 16) * 16 + 16
    w_s = SGPRS_PER_SIMD // sg_alloc
    w = min(MAX_WAVES_PER_SIMD, w_v, w_s, int(res.get("occ", MAX_WAVES_PER_SIMD)))
    b_waves = (w * SIMDS_PER_CU) // waves_block
    b_lds = LDS_PER_CU // max(1, int(res.get("lds", 0)))
    b_threads = (MAX_WAVES_PER_SIMD * SIMDS_PER_CU * 64) // threads
    return max(0, min(b_waves, b_lds, b_threads))


def shared_grid_cap(cus: int, bpc: int, share: int) -> int:
    """Blocks per launch for ``share`` ranks on one GPU of ``cus`` CUs whose kernel fits ``bpc``
    blocks per CU (half the resident capacity split between the ranks, at least 1 block)."""
    if share <= 1:
        return MAX_BLOCKS
    return max(1, min(MAX_BLOCKS, cus * max(1, bpc) // (2 * share)))


_TABLE: Optional[Dict[Tuple[str, Tuple[int, ...]], Dict[str, int]]] = None


def _table_path() -> str:
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_native",
                        "ipc_kernel_resources.json")


def load_table(path: Optional[str] = None) -> Dict[Tuple[str, Tuple[int, ...]], Dict[str, int]]:
    """{(kernel base name, template args): resources} from the build's resource table ({} if absent)."""
    global _TABLE
    if _TABLE is not None and path is None:
        return _TABLE
    out: Dict[Tuple[str, Tuple[int, ...]], Dict[str, int]] = {}
    try:
        with open(path or _table_path()) as f:
            raw = json.load(f)
    except (OSError, ValueError):
        raw = {}
    for name, res in raw.items():
        m = re.search(r"(k_ipc_\w+)(?:<([^>]*)>)?\(", name)
        if not m:
            continue
        args = tuple(int(x) for x in m.group(2).split(",")) if m.group(2) else ()
        out[(m.group(1), args)] = res
    if path is None:
        _TABLE = out
    return out


def table_bpc(family: str, dtype_code: int, dtype_name: str, op_code: int, p: int) -> Optional[int]:
    """Blocks per CU from the compiler resources of the exact kernel instantiation, or None."""
    k = _FAMILY_KERNEL[family]
    if family in ("oneshot", "twoshot", "push", "rs"):
        args: Tuple[int, ...] = (dtype_code, kernel_op(dtype_name, op_code), p)
    elif family == "gather":
        args = (p,)
    elif family == "plan":
        # both pull widths (csrc/runtime/ipc.hip k_ipc_copy_plan<NP>): the cap must hold for either
        got = [load_table().get((k, (w,))) for w in (8, 16)]
        return None if None in got else min(blocks_per_cu(r) for r in got)
    else:
        args = (dtype_code, p)
    res = load_table().get((k, args))
    return None if res is None else blocks_per_cu(res)
