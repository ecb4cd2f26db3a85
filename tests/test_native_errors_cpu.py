"""HIP error hygiene of the native wrapper (CPU, fake library): a failed mp4x HIP call is cleared
from the thread's last-error state before mp4x raises (or, for best-effort release calls, logs),
so PyTorch's next kernel-launch check does not report it as its own failure."""
import pytest

from mp4x.ops import native


class _Lib:
    def __init__(self):
        self.cleared = 0

    def mp4x_clear_error(self):
        self.cleared += 1
        return 1


def test_check_clears_hip_errors_but_not_mp4x_codes(monkeypatch):
    lib = _Lib()
    monkeypatch.setattr(native, "_hip", lib)
    native.check(0, "ok")
    assert lib.cleared == 0
    with pytest.raises(native.NativeError):
        native.check(1, "a hip error")              # hipErrorInvalidValue
    assert lib.cleared == 1
    with pytest.raises(native.NativeError):
        native.check(1001, "mp4x bad argument")     # mp4x's own code: no HIP state to clear
    assert lib.cleared == 1


def test_soft_check_logs_and_clears(monkeypatch, caplog):
    lib = _Lib()
    monkeypatch.setattr(native, "_hip", lib)
    assert native.soft_check(0, "free") == 0 and lib.cleared == 0
    assert native.soft_check(None, "free") is None and lib.cleared == 0   # fake libraries return None
    with caplog.at_level("WARNING"):
        assert native.soft_check(400, "ipc_close_handle") == 400
    assert lib.cleared == 1 and "ipc_close_handle failed" in caplog.text


def test_clear_without_library(monkeypatch):
    monkeypatch.setattr(native, "_hip", None)
    assert native.clear_hip_error() == 0
