"""Control plane: rendezvous, close/exit-code aggregation, failure detection, fault injection.

Reference behaviour: J/rpc/Server.java (rank by sorted "host###port", close codes, heartbeat
and connect timeouts, killMe script), J/comm/ProcessCommSlave.java:143-373 (bootstrap,
exception -> error log + close(1)).
"""
import os
import tempfile
import threading
import time

import numpy as np
import pytest

from harness import run_ranks
from mp4x import CommMaster, Mp4jException, Operands, Operators, ProcessCommSlave
from mp4x.control.client import MasterClient


def _addr_and_rank(comm):
    return comm.transport.address, comm.getRank(), comm.addresses


def test_rank_is_sorted_address_order():
    res, code, _ = run_ranks(4, _addr_and_rank)
    addrs = res[0][2]
    assert addrs == sorted(addrs)
    for r, (addr, rank, _) in res.items():
        assert addrs[rank] == addr
    assert code == 0


def test_requested_ranks_win():
    m = CommMaster(3, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    out = {}

    def reg(rr):
        c = MasterClient("127.0.0.1", m.port)
        out[rr] = c.call("register", f"127.0.0.1###{9000 - rr}", rr)["rank"]

    ths = [threading.Thread(target=reg, args=(r,)) for r in (2, 0, 1)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    assert out == {0: 0, 1: 1, 2: 2}
    # a 4th registration is rejected ("some slave restart, task failed", Server.java:173-176)
    c = MasterClient("127.0.0.1", m.port)
    with pytest.raises(Mp4jException):
        c.call("register", "127.0.0.1###1", -1)
    m.shutdown_server()


def _close_with(comm, bad_rank):
    if comm.getRank() == bad_rank:
        comm.close(3)
    return comm.getRank()


def test_nonzero_close_fails_the_job():
    res, code, _ = run_ranks(3, _close_with, (1,))
    assert code == 1


def test_clean_close_exit_code_zero():
    res, code, _ = run_ranks(3, _close_with, (-1,))
    assert code == 0


def _raise_and_report(comm):
    try:
        raise ValueError("boom")
    except ValueError as e:
        comm.exception(e)   # error log + close(1)
    return comm.getRank()


def test_exception_reports_and_closes_1():
    res, code, _ = run_ranks(2, _raise_and_report)
    assert code == 1


def test_kill_script_and_logs_and_write_file():
    wd = tempfile.mkdtemp()
    m = CommMaster(2, 0, host="127.0.0.1", exit_on_timeout=False, workdir=wd).start()
    comms = [None, None]

    def mk(i):
        comms[i] = ProcessCommSlave("tester", "127.0.0.1", m.port, heartbeat=False)

    ths = [threading.Thread(target=mk, args=(i,)) for i in range(2)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    c0 = next(c for c in comms if c.getRank() == 0)
    c1 = next(c for c in comms if c.getRank() == 1)
    c1.info("not shown (rank-0-only default)")
    c1.info("shown", False)
    c0.info("rank0 says hi")
    c1.error("bad thing")
    c0.writeFile("hello file", "out.txt")
    assert open(os.path.join(wd, "out.txt")).read().strip() == "hello file"
    assert os.path.exists(os.path.join(wd, f"kill_{m.port}.sh"))
    lines = open(os.path.join(wd, f"kill_{m.port}.sh")).read().splitlines()
    assert sum(l.startswith("kill -9") for l in lines) >= 2
    logs = "\n".join(m.logs)
    assert "[rank=1] shown" in logs and "rank0 says hi" in logs and "[rank=1] bad thing" in logs
    assert "not shown" not in logs
    for c in comms:
        c.close(0)
    assert m.stop(timeout=5) == 0


def test_heartbeat_timeout_exit_3():
    m = CommMaster(1, 0, host="127.0.0.1", heartbeat_timeout=0.3, check_interval=0.1, exit_on_timeout=False,
                   workdir=tempfile.mkdtemp()).start()
    c = ProcessCommSlave("t", "127.0.0.1", m.port, heartbeat=False)   # never beats
    time.sleep(0.8)
    assert m.stop(timeout=5) == 3
    c.transport.close()


def test_connect_timeout_exit_2():
    m = CommMaster(2, 0, host="127.0.0.1", connect_timeout=0.3, check_interval=0.1, exit_on_timeout=False,
                   workdir=tempfile.mkdtemp()).start()
    time.sleep(0.8)
    assert m.stop(timeout=5) == 2


def test_heartbeat_keeps_job_alive(monkeypatch):
    import mp4x.parallel.process_comm as pc
    monkeypatch.setattr(pc, "HEARTBEAT_DELAY", 0.05)
    monkeypatch.setattr(pc, "HEARTBEAT_PERIOD", 0.1)
    m = CommMaster(1, 0, host="127.0.0.1", heartbeat_timeout=0.5, check_interval=0.1, exit_on_timeout=False,
                   workdir=tempfile.mkdtemp()).start()
    c = ProcessCommSlave("t", "127.0.0.1", m.port, heartbeat=True)
    time.sleep(1.2)
    assert not m.closed
    c.close(0)
    assert m.stop(timeout=5) == 0


def _faulty(comm):
    a = np.ones(1000)
    for _ in range(3):
        comm.allreduceArray(a, Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0, 1000)
    return "survived"


@pytest.mark.parametrize("p,engine", [(2, "tcp"), (2, "shm"), (3, "shm")])
def test_fault_injection_peer_death_is_detected_not_hung(p, engine):
    # rank 1 dies at its 2nd collective; the others must get a TransportError, not hang.  On
    # /dev/shm the barrier polls the peers' /proc entries, so it fails in well under a second
    # rather than at MP4X_SHM_TIMEOUT (300 s).
    env = {"MP4X_FAULT_INJECT": "1:2:exit", "MP4X_RECV_TIMEOUT": "20"}
    if engine == "tcp":
        env["MP4X_SHM"] = "0"
    t0 = time.monotonic()
    res, code, errs = run_ranks(p, _faulty, expect_fail=True, timeout=60, env=env)
    assert "survived" not in res.values()
    assert errs, "surviving rank should report the failure"
    assert any("closed" in e or "timed out" in e for e in errs)
    if engine == "shm":
        assert any("shared-memory" in e for e in errs)
        assert time.monotonic() - t0 < 20


def test_exchange_pairs_ranks():
    m = CommMaster(2, 0, host="127.0.0.1", exit_on_timeout=False, workdir=tempfile.mkdtemp()).start()
    out = {}

    def go(r):
        out[r] = MasterClient("127.0.0.1", m.port).call("exchange", r)

    ths = [threading.Thread(target=go, args=(r,)) for r in (0, 1)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    assert out == {0: 1, 1: 0}
    m.shutdown_server()
