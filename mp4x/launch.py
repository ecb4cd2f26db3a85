"""Launcher helpers: run the control plane inside a torchrun-style job.

``init_from_env()`` gives every rank a :class:`ProcessCommSlave` without a separately
started master process: rank 0 hosts an embedded :class:`CommMaster` on an ephemeral port
and publishes its address through the launcher's TCPStore (``MASTER_ADDR``/``MASTER_PORT``),
and every rank registers with its launcher rank, so mp4x rank == ``RANK`` == GPU ordinal
``LOCAL_RANK``.  Without launcher variables it builds a single-rank job.

Standalone (reference-style) deployment is still available:
``python -m mp4x.control.master <slaveNum> <port>`` plus ``ProcessCommSlave(login, host, port)``
in every worker.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

from .control.master import CommMaster
from .parallel.process_comm import ProcessCommSlave
from .parallel.thread_comm import ThreadCommSlave

_embedded: Optional[CommMaster] = None


def init_from_env(thread_num: int = 0, heartbeat: bool = True, timeout: float = 600.0):
    """Returns ProcessCommSlave (thread_num == 0) or ThreadCommSlave (thread_num >= 1)."""
    global _embedded
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    key = "mp4x/master_addr"
    host = "127.0.0.1" if os.environ.get("MASTER_ADDR", "127.0.0.1") in ("127.0.0.1", "localhost") \
        else os.environ["MASTER_ADDR"]
    host_master = None
    if world == 1:
        _embedded = host_master = CommMaster(1, 0, host=host, exit_on_timeout=False,
                               heartbeat_timeout=None if heartbeat else float("inf")).start()
        mhost, mport = host, _embedded.port
    else:
        import torch.distributed as dist
        store = dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"]), world,
                              False, timeout=datetime.timedelta(seconds=timeout), wait_for_workers=False)
        if rank == 0:
            os.environ["MP4X_EMBEDDED_MASTER"] = "1"
            bind = "127.0.0.1" if host == "127.0.0.1" else "0.0.0.0"
            _embedded = host_master = CommMaster(world, 0, host=bind, exit_on_timeout=True,
                                   heartbeat_timeout=None if heartbeat else float("inf")).start()
            store.set(key, f"{host}:{_embedded.port}")
        addr = store.get(key).decode()
        mhost, mport = addr.rsplit(":", 1)
        mport = int(mport)
    if thread_num and thread_num >= 1:
        comm = ThreadCommSlave("mp4x", thread_num, mhost, mport, rank=rank, heartbeat=heartbeat)
        pc = comm.processCommSlave
    else:
        comm = pc = ProcessCommSlave("mp4x", mhost, mport, rank=rank, heartbeat=heartbeat)
    if host_master is not None:
        # this process hosts the master: its close() must outlive every other rank's close
        pc._embedded_master = host_master
    return comm


def embedded_master() -> Optional[CommMaster]:
    return _embedded
