"""Host data plane: a persistent TCP full mesh between the ranks.

Replaces the reference's per-message sockets (``getSendDataSocket`` opens a NEW
connection for every message, ProcessCommSlave.java:391-425, with one send and
one receive daemon thread draining BlockingDeques, :71-127).  Here:

* every ordered pair (i → j) uses ONE persistent connection, opened lazily on
  first send (retry loop like the reference's 50 × 30 ms, but time-bounded);
* each incoming connection has a reader thread that drains frames into a
  mailbox keyed by ``(src, tag)``, so a sender never blocks on a slow
  consumer and messages of a later collective may arrive early;
* frames are ``u64 tag | u64 nbytes | body``; bodies are sent zero-copy from
  numpy buffers (``sendall(memoryview)``) and forwarded verbatim by ring
  algorithms without re-encoding.

This is the transport for host-resident data (numpy / Python objects, the
no-GPU configuration).  Device tensors never touch it: they move over RCCL /
xGMI (``device_engine``).
"""
from __future__ import annotations

import os
import socket
import struct
import threading
import time
from collections import deque
from typing import Dict, List, Optional, Sequence, Tuple

from ..exceptions import TransportError
from ..control.protocol import recv_exact

_HDR = struct.Struct("<QQ")
_HELLO = struct.Struct("<Qq")
_MAGIC = 0x6D7034785F746370  # "mp4x_tcp"

SOCK_BUF = int(os.environ.get("MP4X_SOCK_BUF", 8 << 20))


def _tune(s: socket.socket) -> None:
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    for opt in (socket.SO_SNDBUF, socket.SO_RCVBUF):
        try:
            s.setsockopt(socket.SOL_SOCKET, opt, SOCK_BUF)
        except OSError:
            pass


class HostTransport:
    def __init__(self, bind_host: str = "0.0.0.0", advertise_host: Optional[str] = None):
        self._lsock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._lsock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._lsock.bind((bind_host, 0))
        self._lsock.listen(256)
        self.port = self._lsock.getsockname()[1]
        self.advertise_host = advertise_host or "127.0.0.1"
        self.rank = -1
        self.addresses: List[Tuple[str, int]] = []
        self._out: Dict[int, socket.socket] = {}
        self._out_locks: Dict[int, threading.Lock] = {}
        self._out_guard = threading.Lock()
        self._box: Dict[Tuple[int, int], deque] = {}
        self._cv = threading.Condition()
        self._eof: set = set()
        self._closing = False
        self._broken: Optional[str] = None
        self._readers: List[threading.Thread] = []
        self._in_socks: List[socket.socket] = []
        self.bytes_sent = 0
        self.bytes_recv = 0
        self.connect_timeout = float(os.environ.get("MP4X_CONNECT_PEER_TIMEOUT", 120.0))
        self.recv_timeout = float(os.environ.get("MP4X_RECV_TIMEOUT", 0)) or None
        self._acceptor = threading.Thread(target=self._accept_loop, daemon=True, name="mp4x-accept")
        self._acceptor.start()

    # "host###port" string registered at the master (reference format, ProcessCommSlave.java:157)
    @property
    def address(self) -> str:
        return f"{self.advertise_host}###{self.port}"

    def set_peers(self, rank: int, addresses: Sequence[str]) -> None:
        self.rank = rank
        out = []
        for a in addresses:
            h, p = a.rsplit("###", 1)
            out.append((h, int(p)))
        self.addresses = out

    # ----------------------------------------------------------------- inbound
    def _accept_loop(self):
        while True:
            try:
                conn, _ = self._lsock.accept()
            except OSError:
                return
            _tune(conn)
            t = threading.Thread(target=self._reader, args=(conn,), daemon=True, name="mp4x-reader")
            self._in_socks.append(conn)
            self._readers.append(t)
            t.start()

    def _reader(self, conn: socket.socket):
        src = -1
        try:
            magic, src = _HELLO.unpack(recv_exact(conn, _HELLO.size))
            if magic != _MAGIC:
                conn.close()
                return
            while True:
                hdr = conn.recv(_HDR.size, socket.MSG_WAITALL)
                if len(hdr) == 0:
                    break
                if len(hdr) < _HDR.size:
                    hdr += recv_exact(conn, _HDR.size - len(hdr))
                tag, n = _HDR.unpack(hdr)
                body = recv_exact(conn, n) if n else bytearray()
                self.bytes_recv += n
                with self._cv:
                    self._box.setdefault((src, tag), deque()).append(body)
                    self._cv.notify_all()
        except (OSError, ConnectionError) as e:
            if not self._closing:
                with self._cv:
                    self._eof.add(src)
                    self._cv.notify_all()
            return
        with self._cv:
            self._eof.add(src)
            self._cv.notify_all()

    # ----------------------------------------------------------------- outbound
    def _conn(self, dest: int) -> Tuple[socket.socket, threading.Lock]:
        with self._out_guard:
            s = self._out.get(dest)
            if s is not None:
                return s, self._out_locks[dest]
            host, port = self.addresses[dest]
            deadline = time.monotonic() + self.connect_timeout
            while True:
                try:
                    s = socket.create_connection((host, port), timeout=10.0)
                    break
                except OSError as e:
                    if time.monotonic() > deadline:
                        raise TransportError(f"rank {self.rank}: cannot connect to rank {dest} {host}:{port}: {e}")
                    time.sleep(0.03)
            s.settimeout(None)
            _tune(s)
            s.sendall(_HELLO.pack(_MAGIC, self.rank))
            self._out[dest] = s
            self._out_locks[dest] = threading.Lock()
            return s, self._out_locks[dest]

    def send(self, dest: int, tag: int, parts: Sequence) -> int:
        """Send one message made of ``parts`` (bytes / bytearray / memoryview / numpy)."""
        mvs = [memoryview(p).cast("B") if not isinstance(p, (bytes, bytearray)) else p for p in parts]
        n = sum(len(m) for m in mvs)
        if dest == self.rank:
            body = bytearray(n)
            off = 0
            for m in mvs:
                body[off:off + len(m)] = m
                off += len(m)
            with self._cv:
                self._box.setdefault((dest, tag), deque()).append(body)
                self._cv.notify_all()
            return n
        s, lock = self._conn(dest)
        try:
            with lock:
                if n < 65536:
                    s.sendall(_HDR.pack(tag, n) + b"".join(bytes(m) for m in mvs))
                else:
                    s.sendall(_HDR.pack(tag, n))
                    for m in mvs:
                        if len(m):
                            s.sendall(m)
        except OSError as e:
            raise TransportError(f"rank {self.rank}: send to {dest} failed: {e}") from e
        self.bytes_sent += n
        return n

    def recv(self, src: int, tag: int, timeout: Optional[float] = None) -> bytearray:
        key = (src, tag)
        timeout = timeout if timeout is not None else self.recv_timeout
        deadline = None if timeout is None else time.monotonic() + timeout
        with self._cv:
            while True:
                q = self._box.get(key)
                if q:
                    body = q.popleft()
                    if not q:
                        del self._box[key]
                    return body
                if src in self._eof:
                    raise TransportError(f"rank {self.rank}: connection from rank {src} closed while waiting (tag {tag})")
                if self._broken:
                    raise TransportError(self._broken)
                rem = None if deadline is None else deadline - time.monotonic()
                if rem is not None and rem <= 0:
                    raise TransportError(f"rank {self.rank}: recv from {src} tag {tag} timed out")
                self._cv.wait(rem if rem is not None else 5.0)

    def abort(self, why: str) -> None:
        with self._cv:
            self._broken = why
            self._cv.notify_all()

    def close(self) -> None:
        self._closing = True
        try:
            self._lsock.close()
        except OSError:
            pass
        with self._out_guard:
            for s in self._out.values():
                try:
                    s.shutdown(socket.SHUT_RDWR)
                except OSError:
                    pass
                try:
                    s.close()
                except OSError:
                    pass
            self._out.clear()
        for s in self._in_socks:
            try:
                s.close()
            except OSError:
                pass
