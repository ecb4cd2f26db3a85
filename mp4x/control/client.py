"""Slave-side stub of the master protocol (reference: Hadoop ``RPC.getProxy(IServer)``,
/root/reference/src/main/java/com/fenbi/mp4j/comm/ProcessCommSlave.java:151)."""
from __future__ import annotations

import socket
import threading
import time

from ..exceptions import TransportError, Mp4jException
from .protocol import recv_frame, send_frame


class MasterClient:
    def __init__(self, host: str, port: int, connect_timeout: float = 120.0):
        self.host = host
        self.port = int(port)
        self._lock = threading.Lock()
        deadline = time.monotonic() + connect_timeout
        last = None
        while True:
            try:
                s = socket.create_connection((host, self.port), timeout=10.0)
                break
            except OSError as e:
                last = e
                if time.monotonic() > deadline:
                    raise TransportError(f"cannot connect to master {host}:{port}: {e}") from e
                time.sleep(0.05)
        s.settimeout(None)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._sock = s
        self._closed = False

    def call(self, method: str, *args):
        with self._lock:
            if self._closed:
                raise TransportError("master client closed")
            try:
                send_frame(self._sock, {"m": method, "a": list(args)})
                rep = recv_frame(self._sock)
            except (OSError, ConnectionError) as e:
                raise TransportError(f"master rpc {method} failed: {e}") from e
        if "e" in rep:
            raise Mp4jException(f"master rpc {method}: {rep['e']}")
        return rep.get("r")

    def close(self):
        with self._lock:
            if not self._closed:
                self._closed = True
                try:
                    self._sock.close()
                except OSError:
                    pass
