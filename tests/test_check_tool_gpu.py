"""The check CLI on MI355X tensors (``--device cuda``) in process AND thread mode: master +
2 slave processes sharing cuda:0 (gloo stands in for RCCL there; the IPC kernels and the K1
thread-phase kernel run for real).  Reference: CommCheckTool + Thread*Check / Process*Check."""
import os
import subprocess
import sys

import pytest

from test_check_tool import ROOT, _free_port

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode,threads", [("process", 1), ("thread", 2)])
def test_check_tool_device_cuda(tmp_path, mode, threads):
    p = 2
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, MP4X_EXCEPTION_SLEEP="0.1", MP4X_MASTER_BIND="127.0.0.1",
               MP4X_DEVICE_BACKEND="gloo", MP4X_DEVICE_INDEX="0")
    master = subprocess.Popen([sys.executable, "-m", "mp4x.control.master", str(p), str(port)], cwd=tmp_path,
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    slaves = [subprocess.Popen([sys.executable, "-m", "mp4x.check", "tester", "127.0.0.1", str(port), "4099", "20",
                                "1", str(threads), mode, "false", "true", "--device", "cuda"], cwd=tmp_path, env=env,
                               stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for _ in range(p)]
    try:
        outs = [s.communicate(timeout=240)[0] for s in slaves]
        mout = master.communicate(timeout=60)[0]
    finally:
        for x in slaves + [master]:
            if x.poll() is None:
                x.kill()
    assert all(s.returncode == 0 for s in slaves), "\n".join(o[-3000:] for o in outs)
    assert master.returncode == 0, mout[-3000:]
    assert "checks passed" in mout
