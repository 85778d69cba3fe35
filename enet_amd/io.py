"""Batched UDP I/O for the datagram path.

Thin ctypes wrappers over enet_rc_socket_receive_batch / _send_batch
(enet_amd/csrc/rc_io.c: recvmmsg / sendmmsg, the batched form of
enet_socket_receive / enet_socket_send, unix.c:440-528).  Buffers are numpy
arrays; pass a view of pinned memory (``torch.empty(..., pin_memory=True)
.numpy()``) to receive straight into the staging that is copied to the GPU.
"""
from __future__ import annotations

import ctypes as C
import socket as _socket
import struct

import numpy as np

from ._lib import get_lib


class ENetAddress(C.Structure):
    """enet.h:85-89: host = IPv4 address in network byte order, port in host order."""
    _fields_ = [("host", C.c_uint32), ("port", C.c_uint16)]


def address(ip: str, port: int) -> ENetAddress:
    return ENetAddress(struct.unpack("<I", _socket.inet_aton(ip))[0], port)


def receive_batch(fd: int, buf: np.ndarray, slot: int = 4096, max_datagrams: int = 256):
    """Receives up to max_datagrams queued datagrams into buf[i * slot:]; returns
    (count, lengths[count], [(ip, port)] * count).  Non-blocking (0 if none)."""
    assert buf.dtype == np.uint8 and buf.flags.c_contiguous and buf.size >= slot * max_datagrams
    lens = np.zeros(max_datagrams, np.uint32)
    addrs = (ENetAddress * max_datagrams)()
    n = get_lib().enet_rc_socket_receive_batch(fd, buf.ctypes.data_as(C.c_void_p), slot, max_datagrams,
                                               lens.ctypes.data_as(C.c_void_p), C.cast(addrs, C.c_void_p))
    if n < 0:
        raise OSError("enet_rc_socket_receive_batch failed")
    peers = [(_socket.inet_ntoa(struct.pack("<I", addrs[i].host)), int(addrs[i].port)) for i in range(n)]
    return n, lens[:n].copy(), peers


def send_batch(fd: int, datagrams, dest) -> int:
    """Sends every datagram (bytes) to dest (one (ip, port) or a list of them);
    returns how many went out."""
    n = len(datagrams)
    if n == 0:
        return 0
    ln = np.array([len(d) for d in datagrams], np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
    blob = np.frombuffer(b"".join(datagrams) + b"\0", np.uint8)
    if isinstance(dest, tuple):
        dest = [dest] * n
    addrs = (ENetAddress * n)(*[address(ip, port) for ip, port in dest])
    r = get_lib().enet_rc_socket_send_batch(fd, blob.ctypes.data_as(C.c_void_p), off.ctypes.data_as(C.c_void_p),
                                            ln.ctypes.data_as(C.c_void_p), C.cast(addrs, C.c_void_p), n)
    if r < 0:
        raise OSError("enet_rc_socket_send_batch failed")
    return r
