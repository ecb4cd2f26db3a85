"""ctypes binding of the in-tree native libraries (``mp4x/_native``).

``libmp4x_hip.so`` holds the hand-written CDNA4 kernels (csrc/kernels) and the device
runtime (csrc/runtime).  It links against the libamdhip64 that PyTorch-ROCm ships, and
torch is imported before it is loaded, so both share ONE HIP runtime: torch stream
handles and device pointers are passed straight through.

On a GPU box a missing/unloadable library is an error (``NativeUnavailable``), never a
silent fallback: every device collective that needs a kernel goes through here.
"""
from __future__ import annotations

import ctypes
import logging
import os
import threading
from typing import Sequence

from ..exceptions import NativeError, Mp4jException

_HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE_DIR = os.path.join(os.path.dirname(_HERE), "_native")
# MP4X_NATIVE_DEBUG=1: the -DMP4X_DEBUG build with device-side bounds asserts
HIP_LIB = os.path.join(NATIVE_DIR, "libmp4x_hip_debug.so" if os.environ.get("MP4X_NATIVE_DEBUG") == "1"
                       else "libmp4x_hip.so")
HOST_LIB = os.path.join(NATIVE_DIR, "libmp4x_host.so")

c_void_p, c_int, c_int64, c_double, c_size_t = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double, ctypes.c_size_t
PP = ctypes.POINTER(ctypes.c_void_p)


class NativeUnavailable(Mp4jException):
    pass


_lock = threading.RLock()    # launch_ext() calls hip() under it
_hip = None
_host = None

_HIP_SIGS = {
    "mp4x_reduce": (c_int, [c_int, c_int, c_void_p, PP, c_int, c_int64, c_void_p]),
    "mp4x_reduce_strided": (c_int, [c_int, c_int, c_void_p, c_void_p, c_int64, c_int, c_int64, c_void_p]),
    "mp4x_scale": (c_int, [c_int, c_void_p, c_void_p, c_double, c_int64, c_void_p]),
    "mp4x_segment_copy": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int64, c_void_p]),
    "mp4x_gather_rows": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_void_p]),
    "mp4x_quant_fp8": (c_int, [c_int, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "mp4x_dequant_reduce_fp8": (c_int, [c_int, c_void_p, PP, PP, c_int, c_int64, c_int, c_void_p, c_void_p, c_void_p]),
    "mp4x_dequant_fp8": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_int64, c_void_p]),
    "mp4x_zs_temp_bytes": (c_size_t, [c_int64]),
    "mp4x_zs_set_twopass": (c_int, [c_int]),
    "mp4x_zs_encode": (c_int, [c_int, c_void_p, c_void_p, c_int, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_size_t, c_void_p]),
    "mp4x_zs_decode": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int64, c_void_p, c_void_p,
                               c_void_p, c_size_t, c_void_p]),
    "mp4x_key_owner": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p]),
    "mp4x_sort_pairs_temp_bytes": (c_size_t, [c_int64, c_int]),
    "mp4x_sort_pairs_i64": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p, c_size_t, c_void_p]),
    "mp4x_sort_pairs_i64_ex": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_int, c_void_p,
                                       c_size_t, c_void_p]),
    "mp4x_sort_pairs_i32key": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p, c_size_t, c_void_p]),
    "mp4x_partition_pack_scratch_bytes": (c_size_t, [c_int64, c_int]),
    "mp4x_partition_pack": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "mp4x_partition_pack_count": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "mp4x_partition_pack_scatter": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int, c_void_p, c_int, c_void_p,
                                            c_void_p, c_void_p, c_size_t, c_void_p]),
    "mp4x_rle_temp_bytes": (c_size_t, [c_int64]),
    "mp4x_run_starts": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "mp4x_segment_reduce_rows": (c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64,
                                         c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "mp4x_stage_split": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p]),
    "mp4x_keys_from16": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "mp4x_hash_rbk_scratch_bytes": (c_size_t, [c_int64]),
    "mp4x_hash_rbk_supported": (c_int, [c_int, c_int]),
    "mp4x_hash_reduce_by_key": (c_int, [c_int, c_int, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_size_t,
                                        c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "mp4x_dense_rbk_scratch_bytes": (c_size_t, [c_int64, c_int64]),
    "mp4x_dense_reduce_by_key": (c_int, [c_int, c_int, c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int64, c_int64,
                                         c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "mp4x_set_k1_variant": (None, [c_int]),
    "mp4x_set_dq_unroll": (None, [c_int]),
    "mp4x_set_codec_grid": (None, [c_int]),
    "mp4x_set_k1_grid": (None, [c_int64]),
    "mp4x_version": (ctypes.c_char_p, []),
    "mp4x_clear_error": (c_int, []),
    "mp4x_device_count": (c_int, []),
}

_OPTIONAL = set()


def _bind(lib, sigs):
    for name, (res, args) in sigs.items():
        try:
            f = getattr(lib, name)
        except AttributeError:
            if name in _OPTIONAL:
                continue
            raise
        f.restype = res
        f.argtypes = args


def register_signatures(sigs: dict, optional: bool = False) -> None:
    """Extra modules (device runtime) add their C signatures here before first load."""
    _HIP_SIGS.update(sigs)
    if optional:
        _OPTIONAL.update(sigs.keys())
    if _hip is not None:
        _bind(_hip, sigs)


def hip():
    """Load libmp4x_hip.so (after torch, to share its HIP runtime)."""
    global _hip
    if _hip is not None:
        return _hip
    with _lock:
        if _hip is None:
            import torch  # noqa: F401  -- must be loaded first (shared libamdhip64)
            if not os.path.exists(HIP_LIB):
                raise NativeUnavailable(f"{HIP_LIB} not built: run `python tools/build_native.py`")
            lib = ctypes.CDLL(HIP_LIB, mode=ctypes.RTLD_GLOBAL)
            _bind(lib, _HIP_SIGS)
            _hip = lib
    return _hip


def host():
    global _host
    if _host is not None:
        return _host
    with _lock:
        if _host is None:
            if not os.path.exists(HOST_LIB):
                raise NativeUnavailable(f"{HOST_LIB} not built: run `python tools/build_native.py`")
            _host = ctypes.CDLL(HOST_LIB)
            from .host_sigs import HOST_SIGS
            _bind(_host, HOST_SIGS)
    return _host


_team_ext = None


def team_ext():
    """The CPython binding of the host thread team (``_mp4x_team``, csrc/pyext/team_ext.cpp), or
    None when it is not built (ThreadCommSlave then calls the team through ctypes)."""
    global _team_ext
    if _team_ext is None:
        try:
            host()              # the extension links libmp4x_host.so: load it first (own lock)
        except Exception:
            pass
        with _lock:
            if _team_ext is None:
                mod = False
                try:
                    if os.environ.get("MP4X_TEAM_EXT", "1") == "0":
                        raise NativeUnavailable("MP4X_TEAM_EXT=0")
                    import importlib.machinery
                    import importlib.util
                    for suf in importlib.machinery.EXTENSION_SUFFIXES:
                        path = os.path.join(NATIVE_DIR, "_mp4x_team" + suf)
                        if os.path.exists(path):
                            spec = importlib.util.spec_from_file_location("_mp4x_team", path)
                            mod = importlib.util.module_from_spec(spec)
                            spec.loader.exec_module(mod)
                            break
                except Exception:
                    mod = False
                _team_ext = mod
    return _team_ext or None


def _load_ext(name: str):
    import importlib.machinery
    import importlib.util
    for suf in importlib.machinery.EXTENSION_SUFFIXES:
        path = os.path.join(NATIVE_DIR, name + suf)
        if os.path.exists(path):
            spec = importlib.util.spec_from_file_location(name, path)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            return mod
    raise NativeUnavailable(f"{name} is not built (python tools/build_native.py)")


_map_ext = None


def map_ext():
    """The native Dict[key, Tensor] -> ids / rows pass (``_mp4x_map``, csrc/pyext/map_ext.cpp),
    or None when it is not built or ``MP4X_MAP_EXT=0`` (the map collectives then take the
    Python form of the same pass)."""
    global _map_ext
    if _map_ext is None:
        with _lock:
            if _map_ext is None:
                mod = False
                if os.environ.get("MP4X_MAP_EXT", "1") != "0":
                    try:
                        import torch  # noqa: F401 — libtorch_python must be loaded first
                        mod = _load_ext("_mp4x_map")
                    except Exception:   # noqa: BLE001
                        mod = False
                _map_ext = mod
    return _map_ext or None


_hostmap_ext = None


def hostmap_ext():
    """The native host-map passes (``_mp4x_hostmap``, csrc/pyext/hostmap_ext.cpp; no torch), or
    None when not built or ``MP4X_MAP_EXT=0``."""
    global _hostmap_ext
    if _hostmap_ext is None:
        with _lock:
            if _hostmap_ext is None:
                mod = False
                if os.environ.get("MP4X_MAP_EXT", "1") != "0":
                    try:
                        mod = _load_ext("_mp4x_hostmap")
                    except Exception:   # noqa: BLE001
                        mod = False
                _hostmap_ext = mod
    return _hostmap_ext or None


_launch_ext = None


def launch_ext():
    """The ctypes-free launcher of the IPC allreduce (``_mp4x_launch``, csrc/pyext/launch_ext.cpp),
    bound to THIS process's libmp4x_hip.so, or None when not built or ``MP4X_LAUNCH_EXT=0``."""
    global _launch_ext
    if _launch_ext is None:
        with _lock:
            if _launch_ext is None:
                mod = False
                if os.environ.get("MP4X_LAUNCH_EXT", "1") != "0":
                    try:
                        lib = hip()
                        mod = _load_ext("_mp4x_launch")
                        mod.bind(ctypes.cast(lib.mp4x_ipc_allreduce_ex2, ctypes.c_void_p).value)
                        fast = getattr(lib, "mp4x_ipc_fast_allreduce", None)
                        if fast is not None and hasattr(mod, "bind_fast"):
                            mod.bind_fast(ctypes.cast(fast, ctypes.c_void_p).value)
                        plan = getattr(lib, "mp4x_ipc_fast_plan", None)
                        if plan is not None and hasattr(mod, "bind_fast_plan"):
                            mod.bind_fast_plan(ctypes.cast(plan, ctypes.c_void_p).value)
                        frs = getattr(lib, "mp4x_ipc_fast_rs", None)
                        if frs is not None and hasattr(mod, "bind_fast_rs"):
                            mod.bind_fast_rs(ctypes.cast(frs, ctypes.c_void_p).value)
                    except Exception:   # noqa: BLE001 — ctypes path stays
                        mod = False
                _launch_ext = mod
    return _launch_ext or None


def available() -> bool:
    try:
        hip()
        return True
    except Exception:
        return False


def clear_hip_error() -> int:
    """Read and clear this thread's last HIP error (0 if none, or if the library is not loaded):
    a HIP call that failed inside mp4x must not stay "last error" for PyTorch's next kernel-launch
    check to report as ITS failure."""
    lib = _hip
    if lib is None:
        return 0
    try:
        return int(lib.mp4x_clear_error())
    except Exception:   # noqa: BLE001 — an older library without the symbol
        return 0


def check(rc: int, where: str) -> None:
    if rc != 0:
        if rc < 1000:
            clear_hip_error()
        msgs = {1001: "bad argument", 1002: "unsupported dtype/op"}
        raise NativeError(where, rc, msgs.get(rc, "hip error"))


def soft_check(rc: int, where: str, log=None) -> int:
    """Best-effort release calls (close a mapping, free a buffer): a failure is logged and the
    HIP error state cleared instead of raised."""
    if rc:
        clear_hip_error()
        (log or logging.getLogger("mp4x.native")).warning("%s failed: hip error %d", where, rc)
    return rc


def ptr_array(ptrs: Sequence[int]):
    arr = (c_void_p * len(ptrs))(*ptrs)
    return ctypes.cast(arr, PP), arr


_current_raw_stream = None
_capturing_fn = None


def capturing_now() -> bool:
    """``torch.cuda.is_current_stream_capturing()`` without its Python wrapper (on every device
    collective's path)."""
    global _capturing_fn
    if _capturing_fn is None:
        import torch
        _capturing_fn = getattr(torch._C, "_cuda_isCurrentStreamCapturing", None) or \
            torch.cuda.is_current_stream_capturing
    return bool(_capturing_fn())


def stream_ptr(stream=None) -> int:
    """hipStream_t of ``stream`` (default: torch's current stream on the current device).  The
    default case is on every launch's path, so it goes straight to torch's raw-stream query
    instead of building a ``torch.cuda.Stream`` object (measured ~4 us per call)."""
    if stream is not None:
        return int(stream.cuda_stream)
    global _current_raw_stream
    if _current_raw_stream is None:
        import torch
        raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        dev = getattr(torch._C, "_cuda_getDevice", None)
        if raw is not None and dev is not None:
            _current_raw_stream = lambda: raw(dev())      # noqa: E731
        else:
            _current_raw_stream = lambda: torch.cuda.current_stream().cuda_stream   # noqa: E731
    return int(_current_raw_stream())
