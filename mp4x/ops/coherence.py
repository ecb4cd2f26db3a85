"""Cross-XCD coherence probe (csrc/runtime/xcd_probe.hip): does the IPC kernels' system-scope
release / acquire pair (csrc/runtime/ipc_common.hpp ``sys_release`` / ``sys_acquire``, the fences
of every ``block_barrier``) make a producer's plain stores visible to a consumer on another XCD of
the same GPU, and does the two-call stale-line probe SEE the failure when a fence is left out?

The per-XCD L2s of one MI355X are not coherent with each other, so this is the same-GPU analogue of
what the zero-copy forms rely on across GPUs (tests/test_coherence_gpu.py).
"""
from __future__ import annotations

import ctypes

from . import native
from .native import c_int, c_int64, c_void_p, check, stream_ptr

native.register_signatures({
    "mp4x_xcd_probe": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, ctypes.c_uint32, ctypes.c_double,
                               c_void_p]),
    "mp4x_ipc_set_debug": (c_int, [c_void_p, ctypes.c_uint32]),
    "mp4x_debug_build": (c_int, []),
})

NO_RELEASE = 1      # kDbgNoRelease: the producer's release fence left out
NO_ACQUIRE = 2      # kDbgNoAcquire: the consumer's acquire fence left out


def xcd_probe(rounds: int = 64, mask: int = 0, region_vecs: int = 256, spin_s: float = 5.0) -> dict:
    """Run the probe on the current device: 8 producer / 8 consumer workgroups, ``rounds`` rounds
    of ``region_vecs`` 16-byte vectors per region.  ``mask``: NO_RELEASE | NO_ACQUIRE.  Returns
    {"stale": vectors read stale over all rounds, "per_consumer", "xcc" (XCC id per block),
    "cross_xcd": consumer and producer on different XCDs for every pair, "timeout", ...}."""
    import torch
    lib = native.hip()
    dev = torch.device("cuda", torch.cuda.current_device())
    data = torch.zeros(8 * region_vecs * 4, dtype=torch.int32, device=dev)
    flags = torch.zeros(512, dtype=torch.int32, device=dev)         # allocator blocks: 512-B aligned
    out = torch.zeros(34, dtype=torch.int32, device=dev)
    check(lib.mp4x_xcd_probe(data.data_ptr(), flags.data_ptr(), out.data_ptr(), int(region_vecs), int(rounds),
                             int(mask), float(spin_s), stream_ptr()), "mp4x_xcd_probe")
    torch.cuda.synchronize(dev)
    o = [int(x) & 0xFFFFFFFF for x in out.cpu().tolist()]
    xcc = o[16:32]
    pairs = [(xcc[(k + 1) & 7], xcc[8 + k]) for k in range(8)]        # (producer's, consumer's)
    return {"stale": sum(o[8:16]), "per_consumer": o[8:16], "xcc": xcc,
            "cross_xcd": all(a != b for a, b in pairs), "timeout": bool(o[32]), "rounds": rounds,
            "vectors_per_round": 8 * region_vecs, "mask": mask}


def debug_build() -> bool:
    """Is the loaded kernel library the MP4X_DEBUG build (MP4X_NATIVE_DEBUG=1)?"""
    return bool(native.hip().mp4x_debug_build())


def set_barrier_debug(inst, flags: int) -> None:
    """Debug build only: leave block_barrier's release (NO_RELEASE) / acquire (NO_ACQUIRE) out in
    every kernel of IPC instance ``inst`` (its own Signal block)."""
    if not debug_build():
        raise RuntimeError("barrier debug flags need the debug build (MP4X_NATIVE_DEBUG=1)")
    check(native.hip().mp4x_ipc_set_debug(inst._sig, int(flags)), "mp4x_ipc_set_debug")
