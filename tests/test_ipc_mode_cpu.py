"""The dmabuf IPC default (VERDICT r5 Next #5): what ``import mp4x`` found is recorded, and a
failed handle export names the cause and the fix instead of falling back silently."""
import mp4x
from mp4x.parallel.ipc import ipc_mode_report


def test_import_records_the_mode_in_effect():
    at = mp4x.IPC_MODE_AT_IMPORT
    assert set(at) == {"env_before_import", "hip_initialized_before_import"}


def test_report_names_the_legacy_mode_and_the_fix(monkeypatch):
    monkeypatch.setattr(mp4x, "IPC_MODE_AT_IMPORT", {"env_before_import": "1", "hip_initialized_before_import": False})
    rep = ipc_mode_report("ipc_get_handle(data): native error 1 hip error")
    assert rep["dmabuf_expected"] is False
    assert "HSA_ENABLE_IPC_MODE_LEGACY=1" in rep["reason"] and "HSA_ENABLE_IPC_MODE_LEGACY=0" in rep["reason"]
    # HIP initialised before import mp4x with the variable unset: the default came too late
    monkeypatch.setattr(mp4x, "IPC_MODE_AT_IMPORT", {"env_before_import": None, "hip_initialized_before_import": True})
    rep = ipc_mode_report("ipc_get_handle(data): native error 1 hip error")
    assert "initialised before `import mp4x`" in rep["reason"]
    # dmabuf requested and still failing: the error itself, flagged as such
    monkeypatch.setattr(mp4x, "IPC_MODE_AT_IMPORT", {"env_before_import": "0", "hip_initialized_before_import": True})
    rep = ipc_mode_report("ipc_open_handle(rank 1): native error 1 hip error")
    assert rep["dmabuf_expected"] is True and "although the dmabuf mode was requested" in rep["reason"]
    assert "reason" not in ipc_mode_report()
