"""Every C entry point the Python layer binds exists in the built HIP libraries (release and the
device-assert debug build) — checked on CPU (the libraries load without a GPU), so a symbol lost in
a refactor of the native sources fails here instead of silently disabling a device tier on the box."""
import ctypes
import importlib
import os

import pytest

torch = pytest.importorskip("torch")

MODULES = ["mp4x.ops.device_ops", "mp4x.parallel.ipc", "mp4x.parallel.order", "mp4x.parallel.vmm", "mp4x.parallel.sparse",
           "mp4x.parallel.zs", "mp4x.utils.topology"]


def _sigs():
    from mp4x.ops import native
    for m in MODULES:
        try:
            importlib.import_module(m)
        except ImportError:
            pass
    return native, dict(native._HIP_SIGS), set(getattr(native, "_OPTIONAL", set()))


@pytest.mark.parametrize("debug", [False, True])
def test_every_bound_symbol_exists(debug):
    native, sigs, optional = _sigs()
    path = native.HIP_LIB.replace("libmp4x_hip.so", "libmp4x_hip_debug.so") if debug else native.HIP_LIB
    if not os.path.exists(path):
        pytest.skip(f"{path} not built")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    missing = sorted(k for k in sigs if k not in optional and not hasattr(lib, k))
    assert not missing, f"{os.path.basename(path)} lacks {missing}"
