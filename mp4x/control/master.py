"""CommMaster — the control-plane daemon.

Capabilities of the reference master (``CommMaster`` + ``rpc/Server``,
/root/reference/src/main/java/com/fenbi/mp4j/comm/CommMaster.java:41-133,
/root/reference/src/main/java/com/fenbi/mp4j/rpc/Server.java:48-525):

* rendezvous + rank assignment by lexicographic sort of ``"host###port"``
  (Server.java:167-222; more than ``slaveNum`` registrations is rejected —
  "some slave restart, task failed", :173-176).  New: a slave may request an
  explicit rank (torchrun-style launchers), which then wins over the sort.
* barrier (Server.java:131-137), pairing ``exchange`` (:358-370)
* heartbeat map + periodic timeout check: waiting for connections longer than
  ``connect_timeout`` → exit 2, a heartbeat gap longer than ``heartbeat_timeout``
  → exit 3 (:140-164)
* remote log sink ``info/debug/error`` (:225-239)
* close aggregation — exit code 0 iff every slave closed with 0; any non-zero
  close stops the master immediately (:243-289)
* ``shutdown`` (:293-299), ``writeFile`` (:302-316), ``killMe`` kill-script
  collection into ``kill_<port>.sh`` (:319-355)
* RPC allreduce of small payloads (:373-514) — here ordered by RANK, not
  arrival order, so non-commutative user operators are deterministic.
* NEW: a tiny key/value store used to bootstrap the device communicator
  (RCCL unique-id / TCPStore address, IPC handles).

It is a thread-per-connection TCP server speaking msgpack frames
(:mod:`mp4x.control.protocol`).  Run standalone with
``python -m mp4x.control.master <slaveNum> <port>`` (exit code = job status)
or embedded in rank 0 (``CommMaster(n).start()``).
"""
from __future__ import annotations

import logging
import os
import socket
import sys
import threading
import time
from typing import Dict, List, Optional

from .protocol import recv_frame, recv_frame_sized, send_frame, local_ip

LOG = logging.getLogger("mp4x.master")

ADDRESS_DELIM = "#@#"


def _envf(name: str, default: float) -> float:
    try:
        return float(os.environ.get(name, default))
    except ValueError:
        return default


class _Barrier:
    """Generation-counting barrier (reusable, like java.util.concurrent.CyclicBarrier)."""

    def __init__(self, n: int):
        self.n = n
        self.count = 0
        self.gen = 0
        self.cv = threading.Condition()
        self.broken = False

    def wait(self, timeout: Optional[float] = None) -> int:
        with self.cv:
            if self.broken:
                raise RuntimeError("barrier broken")
            gen = self.gen
            self.count += 1
            if self.count == self.n:
                self.count = 0
                self.gen += 1
                self.cv.notify_all()
                return gen
            deadline = None if timeout is None else time.monotonic() + timeout
            while self.gen == gen and not self.broken:
                rem = None if deadline is None else deadline - time.monotonic()
                if rem is not None and rem <= 0:
                    raise TimeoutError("barrier timeout")
                self.cv.wait(rem)
            if self.broken:
                raise RuntimeError("barrier broken")
            return gen

    def break_(self):
        with self.cv:
            self.broken = True
            self.cv.notify_all()


class _Gatherer:
    """p-way rendezvous that returns every rank's contribution, ordered by rank."""

    def __init__(self, n: int):
        self.n = n
        self.cv = threading.Condition()
        self.slots: Dict[int, Dict[int, object]] = {}
        self.results: Dict[int, List[object]] = {}
        self.readers: Dict[int, int] = {}
        self.seq: Dict[int, int] = {}

    def contribute(self, rank: int, value, broken: threading.Event):
        with self.cv:
            gen = self.seq.get(rank, 0)
            self.seq[rank] = gen + 1
            slot = self.slots.setdefault(gen, {})
            slot[rank] = value
            if len(slot) == self.n:
                self.results[gen] = [slot[r] for r in range(self.n)]
                self.readers[gen] = self.n
                del self.slots[gen]
                self.cv.notify_all()
            while gen not in self.results:
                if broken.is_set():
                    raise RuntimeError("master shutting down")
                self.cv.wait(1.0)
            out = self.results[gen]
            self.readers[gen] -= 1
            if self.readers[gen] == 0:
                del self.results[gen]
                del self.readers[gen]
            return out


class CommMaster:
    """Control-plane master.  ``CommMaster(slave_num, port).start(); code = master.stop()``."""

    def __init__(self, slave_num: int, port: int = 0, host: Optional[str] = None,
                 connect_timeout: Optional[float] = None, heartbeat_timeout: Optional[float] = None,
                 check_interval: Optional[float] = None, exit_on_timeout: bool = True,
                 workdir: Optional[str] = None):
        if slave_num < 1:
            raise ValueError("slave_num must be >= 1")
        self.slave_num = slave_num
        self.bind_host = host or os.environ.get("MP4X_MASTER_BIND", "0.0.0.0")
        self.requested_port = port
        self.connect_timeout = connect_timeout or _envf("MP4X_CONNECT_TIMEOUT", 7200.0)
        self.heartbeat_timeout = heartbeat_timeout or _envf("MP4X_HEARTBEAT_TIMEOUT", 600.0)
        self.check_interval = check_interval or _envf("MP4X_CHECK_INTERVAL", 30.0)
        self.exit_on_timeout = exit_on_timeout
        self.workdir = workdir or os.getcwd()

        self._lock = threading.Lock()
        self._reg: List[tuple] = []          # (addr, requested_rank)
        self._addresses: Optional[List[str]] = None
        self._reg_cv = threading.Condition(self._lock)
        self._barrier = _Barrier(slave_num)
        self._gather = _Gatherer(slave_num)
        self._exch_cv = threading.Condition()
        self._exch_waiting: Optional[int] = None
        self._exch_result: Dict[int, int] = {}
        self._kv: Dict[str, bytes] = {}
        self._kv_cv = threading.Condition()
        self._heartbeat: Dict[int, float] = {}
        self._kill_scripts: List[str] = []
        self._kill_barrier = _Barrier(slave_num)
        self._closed_cv = threading.Condition()
        self._closed = False
        self._closed_cnt = 0
        self._close_ok = True
        self._status = "WAITING_FOR_CONNECTING"
        self._start_time = time.monotonic()
        self._stop_evt = threading.Event()
        self._sock: Optional[socket.socket] = None
        self._threads: List[threading.Thread] = []
        self.timeout_code: Optional[int] = None
        self.logs: List[str] = []   # remote log history (also emitted through logging)
        self.rpc_bytes: Dict[str, int] = {}   # request bytes received per RPC method
        self._bytes_lock = threading.Lock()

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "CommMaster":
        s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        s.bind((self.bind_host, self.requested_port))
        s.listen(max(64, 4 * self.slave_num))
        self._sock = s
        t = threading.Thread(target=self._accept_loop, name="mp4x-master-accept", daemon=True)
        t.start()
        c = threading.Thread(target=self._timeout_loop, name="mp4x-master-timeout", daemon=True)
        c.start()
        self._threads += [t, c]
        LOG.info("mp4x master listening on %s:%d for %d slaves", self.host, self.port, self.slave_num)
        return self

    @property
    def port(self) -> int:
        return self._sock.getsockname()[1] if self._sock else self.requested_port

    @property
    def host(self) -> str:
        h = self.bind_host
        if h in ("0.0.0.0", ""):
            return local_ip()
        return h

    def getHostName(self) -> str:  # reference CommMaster.getHostName (:93)
        return self.host

    def getHostPort(self) -> int:  # reference CommMaster.getHostPort (:102)
        return self.port

    def stop(self, timeout: Optional[float] = None) -> int:
        """Block until the job is closed (all slaves closed, or one closed non-zero). Returns exit code."""
        with self._closed_cv:
            deadline = None if timeout is None else time.monotonic() + timeout
            while not self._closed:
                rem = None if deadline is None else deadline - time.monotonic()
                if rem is not None and rem <= 0:
                    break
                self._closed_cv.wait(rem if rem is not None else 1.0)
        code = self.timeout_code if self.timeout_code is not None else (0 if self._close_ok else 1)
        self.shutdown_server()
        return code

    def shutdown_server(self) -> None:
        self._stop_evt.set()
        self._barrier.break_()
        self._kill_barrier.break_()
        if self._sock is not None:
            try:
                self._sock.close()
            except OSError:
                pass

    @property
    def closed(self) -> bool:
        return self._closed

    # ------------------------------------------------------------------ server loops
    def _accept_loop(self):
        while not self._stop_evt.is_set():
            try:
                conn, _ = self._sock.accept()
            except OSError:
                return
            conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            threading.Thread(target=self._serve, args=(conn,), daemon=True, name="mp4x-master-conn").start()

    def _serve(self, conn: socket.socket):
        try:
            while not self._stop_evt.is_set():
                try:
                    req, nb = recv_frame_sized(conn)
                except (ConnectionError, OSError):
                    return
                m = req.get("m")
                with self._bytes_lock:          # control-plane load per method (rpc_stats)
                    self.rpc_bytes[str(m)] = self.rpc_bytes.get(str(m), 0) + nb
                args = req.get("a", [])
                fn = getattr(self, "rpc_" + str(m), None)
                if fn is None:
                    send_frame(conn, {"e": f"unknown method {m}"})
                    continue
                try:
                    res = fn(*args)
                    send_frame(conn, {"r": res})
                except Exception as e:  # report to caller, keep serving
                    LOG.debug("rpc %s failed: %r", m, e)
                    try:
                        send_frame(conn, {"e": f"{type(e).__name__}: {e}"})
                    except OSError:
                        return
        finally:
            try:
                conn.close()
            except OSError:
                pass

    def _timeout_loop(self):
        while not self._stop_evt.wait(self.check_interval):
            now = time.monotonic()
            if self._status == "WAITING_FOR_CONNECTING":
                if now - self._start_time > self.connect_timeout:
                    LOG.error("waiting for connecting timeout > %ss, master will be shut down", self.connect_timeout)
                    self._timeout_exit(2)
                    return
            else:
                for r, t in list(self._heartbeat.items()):
                    if now - t > self.heartbeat_timeout:
                        LOG.error("heartbeat of rank %d timeout > %ss, master will be shut down", r,
                                  self.heartbeat_timeout)
                        self._timeout_exit(3)
                        return

    def _timeout_exit(self, code: int):
        self.timeout_code = code
        with self._closed_cv:
            self._closed = True
            self._close_ok = False
            self._closed_cv.notify_all()
        if self.exit_on_timeout and threading.current_thread() is not threading.main_thread():
            # fail-stop like the reference's System.exit(2/3)
            if os.environ.get("MP4X_MASTER_NO_EXIT") != "1":
                os._exit(code)

    # ------------------------------------------------------------------ RPC methods
    def rpc_register(self, addr: str, requested_rank: int = -1):
        """Reference: ``getAllSlavesInfo`` (Server.java:167-222)."""
        with self._reg_cv:
            if len(self._reg) >= self.slave_num:
                LOG.error("more than %d slaves connecting master, may be some slave restart, task failed!",
                          self.slave_num)
                raise RuntimeError("more than slaveNum slaves registered (slave restart?)")
            self._reg.append((addr, int(requested_rank)))
            LOG.info("connecting: %s, connected count: %d", addr, len(self._reg))
            if len(self._reg) == self.slave_num:
                reqs = [r for _, r in self._reg]
                if all(r >= 0 for r in reqs) and sorted(reqs) == list(range(self.slave_num)):
                    order = sorted(self._reg, key=lambda x: x[1])
                else:
                    order = sorted(self._reg, key=lambda x: x[0])
                self._addresses = [a for a, _ in order]
                now = time.monotonic()
                for r in range(self.slave_num):
                    self._heartbeat[r] = now
                self._status = "WAITING_FOR_HEARTBEAT"
                self._reg_cv.notify_all()
            while self._addresses is None:
                if self._stop_evt.is_set():
                    raise RuntimeError("master stopped")
                self._reg_cv.wait(1.0)
            # rank = position of this registration in the final order
            idx = [i for i, a in enumerate(self._addresses) if a == addr]
            if len(idx) != 1:
                raise RuntimeError(f"duplicate slave address {addr}")
            return {"rank": idx[0], "addresses": list(self._addresses)}

    def rpc_barrier(self, rank: int = -1):
        self._barrier.wait()
        return True

    def rpc_heartbeat(self, rank: int):
        self._heartbeat[int(rank)] = time.monotonic()
        return True

    def _log(self, level: int, rank: int, text: str):
        self.logs.append(text)
        if len(self.logs) > 10000:
            del self.logs[:5000]
        LOG.log(level, "%s", text)

    def rpc_info(self, rank: int, text: str):
        self._log(logging.INFO, rank, text)
        return True

    def rpc_debug(self, rank: int, text: str):
        self._log(logging.DEBUG, rank, text)
        return True

    def rpc_error(self, rank: int, text: str):
        self._log(logging.ERROR, rank, text)
        return True

    def rpc_close(self, rank: int, code: int):
        """Reference: Server.close (:243-272)."""
        LOG.info("recv close message from the slave rank:%s, code:%s", rank, code)
        with self._closed_cv:
            self._close_ok = self._close_ok and (int(code) == 0)
            if int(code) != 0:
                LOG.info("unnormally closed, rank=%s, code:%s", rank, code)
                self._closed = True
                self._closed_cv.notify_all()
                return True
            self._closed_cnt += 1
            if self._closed_cnt >= self.slave_num:
                self._closed = True
                self._closed_cv.notify_all()
                LOG.info("all slaves have sent close messages! server will be closed right now!")
        return True

    def rpc_is_closed(self):
        return {"closed": self._closed, "ok": self._close_ok}

    def rpc_shutdown(self, code: int, message: str):
        """Reference: Server.shutdown (:293-299) — a slave asks the master to exit."""
        LOG.info("%s", message)
        LOG.info("shutdown(%s) invoked", code)
        self.timeout_code = int(code)
        with self._closed_cv:
            self._closed = True
            self._close_ok = False
            self._closed_cv.notify_all()
        return True

    def rpc_write_file(self, content: str, file_name: str):
        path = file_name if os.path.isabs(file_name) else os.path.join(self.workdir, file_name)
        with open(path, "w") as f:
            f.write(content + "\n")
        return True

    def rpc_kill_me(self, rank: int, script: str):
        """Reference: Server.killMe (:319-355) — rank 0 writes kill_<port>.sh."""
        with self._lock:
            self._kill_scripts.append(script)
        self._kill_barrier.wait()
        if int(rank) == 0:
            path = os.path.join(self.workdir, f"kill_{self.port}.sh")
            with open(path, "w") as f:
                for line in self._kill_scripts:
                    f.write(line + "\n")
                if os.environ.get("MP4X_EMBEDDED_MASTER") != "1":
                    f.write(f"kill -9 {os.getpid()}\n")
        return True

    def rpc_exchange(self, rank: int):
        """Pair two arriving ranks (reference Exchanger-based ``exchange``, Server.java:358-370)."""
        with self._exch_cv:
            if self._exch_waiting is None:
                self._exch_waiting = int(rank)
                deadline = time.monotonic() + 3600.0
                while int(rank) not in self._exch_result:
                    rem = deadline - time.monotonic()
                    if rem <= 0:
                        self._exch_waiting = None
                        raise TimeoutError("exchange timeout")
                    self._exch_cv.wait(min(rem, 1.0))
                return self._exch_result.pop(int(rank))
            other = self._exch_waiting
            self._exch_waiting = None
            self._exch_result[other] = int(rank)
            self._exch_cv.notify_all()
            return other

    def rpc_rpc_allreduce(self, rank: int, payload: bytes):
        """Gather every rank's payload (rank order) and return the list to all (Server.java:373-514)."""
        return self._gather.contribute(int(rank), payload, self._stop_evt)

    def rpc_allgather_obj(self, rank: int, payload):
        return self._gather.contribute(int(rank), payload, self._stop_evt)

    def rpc_stats(self):
        """Request bytes the master received per RPC method (control-plane load)."""
        with self._bytes_lock:
            return dict(self.rpc_bytes)

    def rpc_kv_set(self, key: str, value: bytes):
        with self._kv_cv:
            self._kv[key] = value
            self._kv_cv.notify_all()
        return True

    def rpc_kv_get(self, key: str, timeout: float = 600.0):
        deadline = time.monotonic() + float(timeout)
        with self._kv_cv:
            while key not in self._kv:
                rem = deadline - time.monotonic()
                if rem <= 0:
                    raise TimeoutError(f"kv_get({key}) timeout")
                self._kv_cv.wait(min(rem, 1.0))
            return self._kv[key]

    def rpc_status(self):
        return {"status": self._status, "slave_num": self.slave_num, "closed": self._closed}


def main(argv=None) -> int:
    """``python -m mp4x.control.master <slaveNum> <port>`` (reference CommMaster.main, :106-132)."""
    argv = list(sys.argv[1:] if argv is None else argv)
    if len(argv) < 2:
        print("Usage: python -m mp4x.control.master <slaveNum> <port>", file=sys.stderr)
        return 2
    # stdout + log/master{,_warn,_error}.log daily-rolling, or MP4X_LOG_CONFIG (reference:
    # config/log4j_master.properties)
    from ..utils.logconf import configure_logging
    configure_logging("master")
    slave_num, port = int(argv[0]), int(argv[1])
    m = CommMaster(slave_num, port).start()
    print(f"mp4x master {m.host}:{m.port} slaveNum={slave_num}", flush=True)
    code = m.stop()
    LOG.info("master exit code %d", code)
    return code


if __name__ == "__main__":
    sys.exit(main())
