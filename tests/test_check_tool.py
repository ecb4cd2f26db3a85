"""End-to-end CLI: `python -m mp4x.control.master` + `python -m mp4x.check` slaves
(reference: CommMaster.main + CommCheckTool + bin/comm_cluster_error_check.sh)."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("mode,p,threads,compress", [("process", 3, 1, "false"), ("thread", 2, 2, "false"),
                                                     ("process", 2, 1, "true"), ("thread", 2, 3, "true")])
def test_master_and_check_tool_cli(tmp_path, mode, p, threads, compress):
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, MP4X_EXCEPTION_SLEEP="0.1", MP4X_MASTER_BIND="127.0.0.1")
    master = subprocess.Popen([sys.executable, "-m", "mp4x.control.master", str(p), str(port)], cwd=tmp_path,
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    slaves = [subprocess.Popen([sys.executable, "-m", "mp4x.check", "tester", "127.0.0.1", str(port), "5000", "50",
                                "2", str(threads), mode, compress, "true"], cwd=tmp_path, env=env,
                               stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for _ in range(p)]
    try:
        outs = [s.communicate(timeout=240)[0] for s in slaves]
        mout = master.communicate(timeout=60)[0]
    finally:
        for x in slaves + [master]:
            if x.poll() is None:
                x.kill()
    assert all(s.returncode == 0 for s in slaves), "\n".join(outs)
    assert master.returncode == 0, mout
    assert "checks passed" in mout
    assert (tmp_path / f"kill_{port}.sh").exists()
    # log4j-equivalent layout: log/master.log (+ _warn / _error), daily rolling
    log = (tmp_path / "log" / "master.log").read_text()
    assert "all slaves have sent close messages" in log and "master exit code 0" in log
    assert (tmp_path / "log" / "master_error.log").exists()
