"""Collective watchdog — fail-stop detection of hung or failed device collectives.

The reference is fail-stop: slave heartbeats and master timeouts (J/rpc/Server.java:140-164,
J/comm/ProcessCommSlave.java:212-227), ``exception()`` → ``close(1)`` (:360-373).  A hang
INSIDE a collective is invisible to that machinery — the heartbeat thread keeps beating
while the main thread sits in a socket read forever.  On MI355X the same happens when a GPU
stream never drains (an RCCL ring or an IPC barrier waiting on a dead or diverged peer).
This watchdog is the missing detector, one daemon thread per device engine:

* host side — every device collective is bracketed (:meth:`begin` / :meth:`end`); a call
  still inside after ``MP4X_WATCHDOG_TIMEOUT`` seconds (default 600, the reference's
  heartbeat gap, Server.java:82-83) is a hang (gloo / p2p / host-synchronising schedules
  block the calling thread);
* device side — when an outermost collective returns and no earlier event is still
  outstanding, a HIP event is recorded on the stream it ran on; an event still pending after
  the timeout means that stream is stuck.  This is the asynchronous-error check
  ``ncclCommGetAsyncError`` polling gives an RCCL job (torch's ProcessGroupNCCL watchdog does it
  for RCCL alone), extended to mp4x's own kernels.  One outstanding event at a time keeps the
  latency tier cheap (a record per watchdog period at most, not per call; measured: a 4 KiB
  public-API allreduce went from 20 to 29 us with an event per call);
* IPC error words — the bounded spins of ``csrc/runtime/ipc.hip`` record a timed-out
  barrier in the signal block and exit; the watchdog reads that word on a private stream
  and treats a set word as a failure: that collective's result is invalid.

On failure, ``MP4X_WATCHDOG_ACTION``:

``exit``  (default) report to the master's error log, send ``close(5)`` (the master turns
          any non-zero close into a failed job, Server.java:252-261) and ``os._exit(5)`` —
          fail-stop, as the reference's ``System.exit`` (the driver tears the RCCL
          communicators down with the process);
``abort`` report and abort the communicators: the blocked call returns with an error and
          every later collective on this rank raises :class:`Mp4jException`;
``log``   report only (the error word is cleared and monitoring continues).

The master is reached through a connection of the watchdog's own: the main thread may hold
the shared client's lock inside a blocked RPC.  ``MP4X_WATCHDOG=0`` disables the thread.
"""
from __future__ import annotations

import collections
import itertools
import logging
import os
import threading
import time
from typing import Callable, Deque, Dict, Optional, Tuple

from ..exceptions import Mp4jException

LOG = logging.getLogger("mp4x.watchdog")

EXIT_CODE = 5   # heartbeat loss exits 4 (reference); a watchdog fail-stop exits 5
ACTIONS = ("exit", "abort", "log")


def enabled() -> bool:
    return os.environ.get("MP4X_WATCHDOG", "1") == "1"


class CollectiveWatchdog:
    def __init__(self, engine=None, timeout: Optional[float] = None, period: Optional[float] = None,
                 action: Optional[str] = None, on_failure: Optional[Callable[[str], None]] = None):
        self.engine = engine
        self.timeout = float(timeout if timeout is not None else os.environ.get("MP4X_WATCHDOG_TIMEOUT", 600.0))
        default_period = min(5.0, max(0.02, self.timeout / 4))
        self.period = float(period if period is not None else os.environ.get("MP4X_WATCHDOG_PERIOD", default_period))
        self.action = (action or os.environ.get("MP4X_WATCHDOG_ACTION", "exit")).lower()
        if self.action not in ACTIONS:
            raise Mp4jException(f"MP4X_WATCHDOG_ACTION must be one of {ACTIONS}, not {self.action!r}")
        self.on_failure = on_failure
        self.failure: Optional[str] = None
        self.paused = 0                      # > 0: skip the IPC error-word check (autotune probes)
        self.quiet = 0                       # > 0: no device API calls at all (hipGraph capture)
        self._lock = threading.Lock()
        self._inflight: Dict[int, Tuple[str, float]] = {}   # GIL-atomic dict ops, no lock
        self._tokens = itertools.count()
        self._pending: Dict[int, Deque] = {}   # stream handle -> deque[(name, t_enqueued, event)]
        self._npending = 0                     # events recorded and not yet seen complete
        self._pool = []                        # completed events, reused
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._loop, daemon=True, name="mp4x-watchdog")
        self._thread.start()

    # ------------------------------------------------------------------ caller side
    def begin(self, name: str) -> int:
        if self.failure is not None and self.action == "abort":
            raise Mp4jException(f"collective watchdog: {self.failure}")
        tok = next(self._tokens)
        self._inflight[tok] = (name, time.monotonic())
        return tok

    def end(self, tok: int, device=None) -> None:
        ent = self._inflight.pop(tok, None)
        if ent is None or self._inflight or self._npending or device is None or \
                getattr(device, "type", None) != "cuda":
            return                       # nested call, or an outstanding event already covers the stream
        import torch
        if torch.cuda.is_current_stream_capturing():
            return                       # graph capture: nothing may be recorded outside the graph
        stream = torch.cuda.current_stream(device)
        with self._lock:
            ev = self._pool.pop() if self._pool else None
        if ev is None:
            ev = torch.cuda.Event()
        ev.record(stream)
        with self._lock:
            self._pending.setdefault(stream.cuda_stream, collections.deque()).append((ent[0], time.monotonic(), ev))
            self._npending += 1

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not threading.current_thread():
            self._thread.join(timeout=max(1.0, 2 * self.period))

    # ------------------------------------------------------------------ watchdog thread
    def _loop(self):
        while not self._stop.wait(self.period):
            try:
                msg = self.check()
            except Exception as e:      # noqa: BLE001 — a failed poll is retried next period
                LOG.debug("watchdog poll failed: %s", e)
                continue
            if msg:
                self._fire(msg)
                if self.action != "log":
                    return

    def check(self) -> Optional[str]:
        """One poll: the failure message, or None."""
        now = time.monotonic()
        inflight = list(self._inflight.values())
        with self._lock:
            streams = list(self._pending.values())
        for name, t0 in inflight:
            if now - t0 > self.timeout:
                return f"{name} blocked on the host for {now - t0:.1f} s (timeout {self.timeout:g} s)"
        if self.quiet:
            # a global-mode graph capture is running: a query or synchronise from this thread
            # would invalidate it, so only the host-side check runs
            return None
        for dq in streams:
            while dq:
                name, t0, ev = dq[0]
                if ev.query():
                    dq.popleft()
                    with self._lock:
                        self._pool.append(ev)
                        self._npending -= 1
                    continue
                if now - t0 > self.timeout:
                    return (f"{name} not complete on the device {now - t0:.1f} s after it was issued "
                            f"(timeout {self.timeout:g} s)")
                break
        if not self.paused:
            err = self._ipc_error()
            if err:
                return (f"IPC barrier timeout (error word {err}): a peer never arrived; the result of that "
                        f"IPC collective is invalid")
        return None

    def _ipc_error(self) -> int:
        eng = self.engine
        if eng is None:
            return 0
        for name in ("_ipc_obj", "_ipc_large", "_ipc_fp8_big"):
            inst = getattr(eng, name, None)
            if inst is not None:
                w = inst.error_word(clear=self.action == "log")
                if w:
                    return w
        return 0

    def _fire(self, msg: str) -> None:
        self.failure = msg
        LOG.error("collective watchdog: %s", msg)
        if self.on_failure is not None:
            self.on_failure(msg)
            return
        comm = getattr(self.engine, "comm", None)
        rank = getattr(comm, "rank", -1)
        cli = None
        try:
            srv = getattr(comm, "server", None)
            if srv is not None:
                from ..control.client import MasterClient
                cli = MasterClient(srv.host, srv.port, connect_timeout=10.0)
                cli.call("error", rank, f"[rank={rank}] collective watchdog: {msg}")
                if self.action == "exit":
                    cli.call("close", rank, EXIT_CODE)
        except Exception as e:          # noqa: BLE001 — the master may be gone as well
            LOG.error("watchdog could not reach the master: %s", e)
        finally:
            if cli is not None:
                cli.close()
        if self.action == "exit":
            # exit first: aborting the communicators would wake the blocked caller, which could
            # then exit on its own (status 0) before this thread gets here
            logging.shutdown()
            os._exit(EXIT_CODE)
        if self.action == "abort":
            try:
                self.engine.abort()
            except Exception as e:      # noqa: BLE001
                LOG.error("watchdog abort failed: %s", e)
