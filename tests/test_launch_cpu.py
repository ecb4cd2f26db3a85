"""The driver's launch path on CPU: ``torch.distributed.run`` with 4 ranks runs ``bench.py --cpu``
(rank 0 embeds the master, gloo stands in for RCCL).  Every rank must exit 0: rank 0 hosts the
master, so its close() has to outlive the other ranks' close messages (a reset connection there
used to fail a finished benchmark)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_torchrun_bench_dry_run_all_ranks_exit_clean(tmp_path):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--cpu", "--gpus", "4", "--steps", "3", "--warmup", "1", "--bytes", "4000000"]
    r = subprocess.run(cmd, cwd=tmp_path, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stdout[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert len(lines) == 1
    rec = lines[0]
    assert rec["n_gpus"] == 4 and rec["steps"] == 3 and rec["value"] > 0
    # value is the per-rank nccl-tests busbw (BASELINE metric), not the whole-job sum
    assert rec["value"] == rec["busbw_gbps_per_rank"]
    assert abs(rec["aggregate_busbw_gbps"] - 4 * rec["busbw_gbps_per_rank"]) < 1e-2
    assert abs(rec["busbw_gbps_per_rank"] - rec["algbw_gbps"] * 2 * 3 / 4) < 1e-2
    assert "e+" not in rec["config"]["model"]
