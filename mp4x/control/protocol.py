"""Wire framing shared by the master (control plane) and the host data plane.

Control messages are msgpack maps in length-prefixed frames::

    u64 little-endian payload length | msgpack payload

A request is ``{"m": method, "a": [args...]}``; a reply is ``{"r": value}`` or
``{"e": "error text"}``.  This replaces the reference's Hadoop-IPC RPC
(``IServer`` protocol, /root/reference/src/main/java/com/fenbi/mp4j/rpc/IServer.java:38-58)
with a dependency-free, language-neutral format.
"""
from __future__ import annotations

import socket
import struct

import msgpack

_LEN = struct.Struct("<Q")
MAX_FRAME = 1 << 40


def recv_exact(sock: socket.socket, n: int) -> bytearray:
    buf = bytearray(n)
    mv = memoryview(buf)
    got = 0
    while got < n:
        # MSG_WAITALL: one syscall for the whole remainder, slept in with the GIL released (the
        # mesh's reader threads then do not contend with the merging thread chunk by chunk)
        r = sock.recv_into(mv[got:], n - got, socket.MSG_WAITALL)
        if r == 0:
            raise ConnectionError("peer closed connection")
        got += r
    return buf


def send_frame(sock: socket.socket, obj) -> None:
    body = msgpack.packb(obj, use_bin_type=True)
    sock.sendall(_LEN.pack(len(body)) + body if len(body) < 65536 else _LEN.pack(len(body)))
    if len(body) >= 65536:
        sock.sendall(body)


def recv_frame(sock: socket.socket):
    return recv_frame_sized(sock)[0]


def recv_frame_sized(sock: socket.socket):
    """(decoded frame, body bytes)."""
    (n,) = _LEN.unpack(recv_exact(sock, _LEN.size))
    if n > MAX_FRAME:
        raise ConnectionError(f"frame too large: {n}")
    return msgpack.unpackb(recv_exact(sock, n), raw=False, strict_map_key=False), n


def local_ip() -> str:
    """Best-effort address other hosts can reach us at (127.0.0.1 when single-host)."""
    import os
    env = os.environ.get("MP4X_HOST")
    if env:
        return env
    try:
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        try:
            s.connect(("10.255.255.255", 1))
            ip = s.getsockname()[0]
        finally:
            s.close()
        return ip
    except OSError:
        return "127.0.0.1"
