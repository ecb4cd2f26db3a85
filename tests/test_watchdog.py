"""Collective watchdog (ncclCommGetAsyncError polling, configurable timeouts,
fail-stop).  Unit tests of the detector plus a real 2-process job on gloo where one rank never
joins a device collective: the blocked rank reports to the master and exits with code 5."""
import threading
import time

import pytest

torch = pytest.importorskip("torch")

from harness import LAST, run_ranks  # noqa: E402
from mp4x import Mp4jException, Operators  # noqa: E402
from mp4x.parallel.watchdog import EXIT_CODE, CollectiveWatchdog  # noqa: E402


def _wait(cond, timeout=5.0):
    t0 = time.monotonic()
    while not cond():
        if time.monotonic() - t0 > timeout:
            return False
        time.sleep(0.01)
    return True


def test_host_hang_is_detected():
    hits = []
    wd = CollectiveWatchdog(None, timeout=0.2, period=0.02, action="abort", on_failure=hits.append)
    try:
        tok = wd.begin("allreduce")
        assert _wait(lambda: hits)
        assert "allreduce blocked on the host" in hits[0]
        wd.end(tok)
        with pytest.raises(Mp4jException, match="collective watchdog"):
            wd.begin("allreduce")          # abort mode: later collectives fail fast
    finally:
        wd.stop()


def test_completed_calls_never_fire():
    hits = []
    wd = CollectiveWatchdog(None, timeout=0.1, period=0.01, action="exit", on_failure=hits.append)
    try:
        for _ in range(50):
            wd.end(wd.begin("reduce_scatter"))
            time.sleep(0.002)
        time.sleep(0.3)
        assert not hits and wd.failure is None
        # nested calls (reduce -> gather) keep the outer one in flight only
        outer = wd.begin("reduce")
        wd.end(wd.begin("gather"))
        wd.end(outer)
        assert not wd._inflight
    finally:
        wd.stop()


class _FakeIpc:
    def __init__(self):
        self.word = 0
        self.cleared = 0

    def error_word(self, clear=False):
        w = self.word
        if clear:
            self.word = 0
            self.cleared += 1
        return w


class _FakeEngine:
    def __init__(self):
        self._ipc_obj = _FakeIpc()
        self._ipc_large = None


def test_ipc_error_word_is_a_failure_unless_paused():
    eng = _FakeEngine()
    hits = []
    wd = CollectiveWatchdog(eng, timeout=60, period=0.01, action="log", on_failure=hits.append)
    try:
        wd.paused += 1                      # autotune probing: expected timeouts are not failures
        eng._ipc_obj.word = 2
        time.sleep(0.1)
        assert not hits
        wd.paused -= 1
        assert _wait(lambda: hits)
        assert "IPC barrier timeout (error word 2)" in hits[0]
        assert eng._ipc_obj.cleared >= 1   # log mode acknowledges the word and keeps watching
    finally:
        wd.stop()


def test_bad_action_rejected():
    with pytest.raises(Mp4jException):
        CollectiveWatchdog(None, timeout=1, period=1, action="explode")


def _hang_job(comm):
    eng = comm.device                      # both ranks bring the gloo communicator up
    assert eng.watchdog is not None
    if comm.getRank() == 0:
        t = torch.ones(64)
        eng.allreduce(t, 0, 64, Operators.Float.SUM)     # rank 1 never joins
        return "returned"
    time.sleep(6.0)
    return "ok"


def test_blocked_rank_fail_stops_with_exit_code_5():
    env = {"MP4X_WATCHDOG_TIMEOUT": "1.5", "MP4X_WATCHDOG_PERIOD": "0.1", "MP4X_DEVICE_BACKEND": "gloo"}
    res, code, errs = run_ranks(2, _hang_job, timeout=60, expect_fail=True, env=env)
    assert 0 not in res                    # rank 0 never returned from the collective
    assert LAST["exitcodes"].count(EXIT_CODE) == 1   # (process order is not rank order)
    assert code != 0                       # the master turned close(5) into a failed job
    assert any("collective watchdog" in line and "allreduce blocked" in line for line in LAST["logs"])


@pytest.mark.gpu
def test_stuck_stream_is_detected_on_device():
    """A kernel that does not finish within the timeout (torch.cuda._sleep) trips the event check."""
    hits = []
    wd = CollectiveWatchdog(None, timeout=0.05, period=0.01, action="log", on_failure=hits.append)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        torch.cuda._sleep(1)                # warm the launch path: the host bracket below stays short
        torch.cuda.synchronize()
        torch.cuda._sleep(500_000_000)      # >= 0.2 s at any shader clock the box runs
        wd.end(wd.begin("allreduce"), dev)  # the stream's event lands behind the long kernel
        assert _wait(lambda: hits, 10.0)
        assert "allreduce not complete on the device" in hits[0]
        torch.cuda.synchronize()
    finally:
        wd.stop()


def test_watchdog_thread_is_daemon_and_stops():
    wd = CollectiveWatchdog(None, timeout=10, period=0.01, action="log")
    assert wd._thread.daemon
    wd.stop()
    assert _wait(lambda: not wd._thread.is_alive(), 2.0)
    assert threading.active_count() >= 1


def test_quiet_skips_device_polls():
    eng = _FakeEngine()
    eng._ipc_obj.word = 1
    hits = []
    wd = CollectiveWatchdog(eng, timeout=60, period=0.01, action="log", on_failure=hits.append)
    try:
        wd.quiet += 1                       # e.g. a hipGraph capture in progress
        time.sleep(0.1)
        assert not hits and eng._ipc_obj.cleared == 0
        wd.quiet -= 1
        assert _wait(lambda: hits)
    finally:
        wd.stop()
