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


def _run(tmp_path, nproc=4, extra_env=None, steps=3):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--cpu", "--gpus", str(nproc), "--steps", str(steps), "--warmup", "1", "--bytes", "4000000"]
    # stderr apart from stdout, as the driver reads it: the ranks' warnings (a failed verification
    # is reported on stderr by every rank) must not interleave with rank 0's JSON lines
    r = subprocess.run(cmd, cwd=tmp_path, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT, **(extra_env or {})))
    r.stdout = r.stdout + r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    return r, lines


def test_torchrun_bench_dry_run_all_ranks_exit_clean(tmp_path):
    r, lines = _run(tmp_path)
    assert r.returncode == 0, r.stdout[-3000:]
    # the verified headline right after its measurement, then the enriched final line (same numbers)
    assert [x["phase"] for x in lines] == ["headline", "final"], lines
    assert lines[0]["value"] == lines[1]["value"] and lines[0]["verified"] is True
    rec = lines[-1]
    assert rec["n_gpus"] == 4 and rec["steps"] == 3 and rec["value"] > 0
    # value is the per-rank nccl-tests busbw (BASELINE metric), not the whole-job sum
    assert rec["value"] == rec["busbw_gbps_per_rank"]
    assert abs(rec["aggregate_busbw_gbps"] - 4 * rec["busbw_gbps_per_rank"]) < 1e-2
    assert abs(rec["busbw_gbps_per_rank"] - rec["algbw_gbps"] * 2 * 3 / 4) < 1e-2
    assert "e+" not in rec["config"]["model"]
    # self-verification of the timed call (exact pattern vs the fp64 answer, MAX over ranks)
    assert rec["verified"] is True and rec["max_abs_err"] == 0.0, rec
    # equal-method RCCL baseline keys (None without RCCL: gloo dry run)
    for k in ("rccl_busbw_gbps", "rccl_p50_ms", "rccl_baseline"):
        assert k in rec
    assert rec["config"]["scale"] == 0.25 and rec["config"]["autotune_iters"] >= 5


def test_bench_values_stay_bounded_over_many_steps(tmp_path):
    # scale=1/p: 60 SUM steps at p=2 would otherwise multiply the data by 2^60
    r, lines = _run(tmp_path, nproc=2, steps=60)
    assert r.returncode == 0, r.stdout[-3000:]
    assert lines[0]["verified"] is True


def test_bench_wrong_result_fails_the_run(tmp_path):
    # a wrong element on one rank (test hook standing in for a broken kernel): verified false, rc != 0
    r, lines = _run(tmp_path, nproc=2, extra_env={"MP4X_BENCH_CORRUPT": "1"})
    assert r.returncode != 0, r.stdout[-3000:]
    assert len(lines) == 2 and all(x["verified"] is False and x["max_abs_err"] >= 1.0 for x in lines), lines


def test_headline_survives_a_hang_after_it(tmp_path):
    """VERDICT r4 Next #3: the headline line is printed right after its measurement; a stage after
    it that never returns (test hook in the extras) and the driver's kill cannot lose it."""
    import signal
    import time
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--cpu", "--gpus", "2", "--steps", "3", "--warmup", "1", "--bytes", "4000000"]
    pr = subprocess.Popen(cmd, cwd=tmp_path, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                          env=dict(os.environ, PYTHONPATH=ROOT, MP4X_BENCH_TEST_HANG="extras",
                                   MP4X_BENCH_TEST_HANG_S="60"),
                          start_new_session=True)
    got = None
    t0 = time.monotonic()
    try:
        for line in pr.stdout:
            if line.startswith('{"metric"'):
                got = json.loads(line)
                break
            if time.monotonic() - t0 > 240:
                break
        time.sleep(1.0)
        assert pr.poll() is None, "the hook should hang the run after the headline"
    finally:
        # what the driver's timeout does: the launcher and every rank it started (the ranks lead
        # process groups of their own, so each is killed by its exact pid)
        import psutil
        try:
            kids = psutil.Process(pr.pid).children(recursive=True)
        except psutil.NoSuchProcess:
            kids = []
        for k in kids:
            try:
                k.kill()
            except psutil.NoSuchProcess:
                pass
        os.killpg(pr.pid, signal.SIGKILL)
        pr.wait(30)
        psutil.wait_procs(kids, timeout=30)
    assert got is not None and got["phase"] == "headline" and got["verified"] is True, got
    assert got["value"] > 0 and got["n_gpus"] == 2
