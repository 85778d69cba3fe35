"""ctypes access to the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Two coders share one interface:
  * ``Coder("port")``      -- oracle/liboracle.so, the C restatement (rc_oracle.c)
  * ``Coder("reference")`` -- oracle/_ref/libenet_ref.so, the real compress.c
                              compiled from /root/reference by oracle/Makefile

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product package (enet_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PORT_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libenet_ref.so")


class _Buf(C.Structure):
    _fields_ = [("data", C.c_void_p), ("dataLength", C.c_size_t)]


_u8p = C.POINTER(C.c_uint8)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


_libs: dict = {}


def _load(path: str) -> C.CDLL:
    if path not in _libs:
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        _libs[path] = C.CDLL(path)
    return _libs[path]


def port_lib() -> C.CDLL:
    lib = _load(PORT_SO)
    lib.or_fnv1a64_packets.restype = C.c_uint64
    lib.or_fnv1a64_packets.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
    lib.cpubench_roundtrip.restype = C.c_int
    lib.cpubench_roundtrip.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_size_t, C.c_int, C.POINTER(C.c_double),
                                       C.POINTER(C.c_double), C.POINTER(C.c_uint64),
                                       C.POINTER(C.c_uint64)]
    return lib


def have_reference() -> bool:
    return os.path.exists(REF_SO)


class Coder:
    """One coder context (compress.c:48-66) of the port or of the reference."""

    def __init__(self, kind: str = "port"):
        if kind == "port":
            lib = _load(PORT_SO)
            names = ("or_create", "or_destroy", "or_compress", "or_decompress")
        elif kind == "reference":
            lib = _load(REF_SO)
            names = ("enet_range_coder_create", "enet_range_coder_destroy",
                     "enet_range_coder_compress", "enet_range_coder_decompress")
        else:
            raise ValueError(kind)
        self.kind = kind
        self._create, self._destroy, self._comp, self._decomp = (getattr(lib, n) for n in names)
        self._create.restype = C.c_void_p
        self._destroy.argtypes = [C.c_void_p]
        self._comp.restype = C.c_size_t
        self._comp.argtypes = [C.c_void_p, C.POINTER(_Buf), C.c_size_t, C.c_size_t, C.c_void_p, C.c_size_t]
        self._decomp.restype = C.c_size_t
        self._decomp.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        self.ctx = self._create()

    def close(self):
        if self.ctx:
            self._destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def compress_gather(self, backing: bytes, spans: Sequence[tuple], in_limit: int,
                        out_limit: int):
        """``spans`` = [(start, length), ...] into ``backing`` (an empty buffer's
        data pointer still points at backing[start], as in compress.c:279-284).
        Returns (return_value, output_bytes)."""
        arr = np.frombuffer(bytes(backing) + b"\0" * 8, dtype=np.uint8).copy()
        base = arr.ctypes.data
        bufs = (_Buf * max(1, len(spans)))()
        for i, (s, l) in enumerate(spans):
            bufs[i].data = base + s
            bufs[i].dataLength = l
        out = np.zeros(max(1, out_limit), dtype=np.uint8)
        r = self._comp(self.ctx, bufs, len(spans), in_limit, _ptr(out), out_limit)
        return int(r), bytes(out[: r])

    def compress(self, data: bytes, out_limit: int | None = None, in_limit: int | None = None):
        if out_limit is None:
            out_limit = 2 * len(data) + 64
        if in_limit is None:
            in_limit = len(data)
        return self.compress_gather(data, [(0, len(data))], in_limit, out_limit)

    def decompress(self, data: bytes, out_limit: int = 4096):
        arr = np.frombuffer(bytes(data) + b"\0", dtype=np.uint8).copy()
        out = np.zeros(max(1, out_limit), dtype=np.uint8)
        r = self._decomp(self.ctx, _ptr(arr), len(data), _ptr(out), out_limit)
        return int(r), bytes(out[: r])


def compress_batch(data: np.ndarray, off: np.ndarray, ln: np.ndarray, kind: str = "port",
                   cap_fn=lambda n: 2 * n + 64):
    """Compresses every packet; returns (out, out_off, out_cap, out_len)."""
    cap = cap_fn(ln.astype(np.uint64)).astype(np.uint32)
    out_off = np.zeros(len(ln), dtype=np.uint64)
    if len(ln) > 1:
        out_off[1:] = np.cumsum(cap[:-1], dtype=np.uint64)
    out = np.zeros(int(cap.sum(dtype=np.uint64)) + 1, dtype=np.uint8)
    out_len = np.zeros(len(ln), dtype=np.uint32)
    if kind == "port":
        lib = port_lib()
        lib.or_compress_batch(_ptr(data), _ptr(off), _ptr(ln), C.c_size_t(len(ln)), _ptr(out),
                              _ptr(out_off), _ptr(cap), _ptr(out_len))
    else:
        c = Coder(kind)
        base = data.ctypes.data
        for i in range(len(ln)):
            buf = (_Buf * 1)()
            buf[0].data = base + int(off[i])
            buf[0].dataLength = int(ln[i])
            out_len[i] = c._comp(c.ctx, buf, 1, int(ln[i]), out.ctypes.data + int(out_off[i]), int(cap[i]))
    return out, out_off, cap, out_len


def decompress_batch(data: np.ndarray, off: np.ndarray, ln: np.ndarray, cap: np.ndarray):
    """Decompresses every packet with the port; returns (out, out_off, out_len)."""
    cap = cap.astype(np.uint32)
    out_off = np.zeros(len(ln), dtype=np.uint64)
    if len(ln) > 1:
        out_off[1:] = np.cumsum(cap[:-1], dtype=np.uint64)
    out = np.zeros(int(cap.sum(dtype=np.uint64)) + 1, dtype=np.uint8)
    out_len = np.zeros(len(ln), dtype=np.uint32)
    port_lib().or_decompress_batch(_ptr(data), _ptr(off), _ptr(ln), C.c_size_t(len(ln)), _ptr(out),
                                   _ptr(out_off), _ptr(cap), _ptr(out_len))
    return out, out_off, out_len


def fnv_digest(out: np.ndarray, out_off: np.ndarray, out_len: np.ndarray) -> str:
    """SURVEY.md §8c batch digest as 16 hex digits."""
    lib = port_lib()
    h = lib.or_fnv1a64_packets(_ptr(out), _ptr(out_off.astype(np.uint64)),
                               _ptr(out_len.astype(np.uint32)), len(out_len))
    return f"{h:016x}"


def cpu_roundtrip(data, off, ln, threads: int, kind: str = "reference"):
    """Times compress then decompress of the whole batch on ``threads`` host
    threads (one context each).  Returns dict(t_compress, t_decompress,
    compressed_bytes, mismatches)."""
    lib = port_lib()
    tc, td = C.c_double(), C.c_double()
    cb, mm = C.c_uint64(), C.c_uint64()
    path = REF_SO.encode() if kind == "reference" else b""
    rc = lib.cpubench_roundtrip(path, _ptr(data), _ptr(off.astype(np.uint64)),
                                _ptr(ln.astype(np.uint32)), len(ln), threads,
                                C.byref(tc), C.byref(td), C.byref(cb), C.byref(mm))
    if rc != 0:
        raise RuntimeError(f"cpubench_roundtrip failed rc={rc}")
    return dict(t_compress=tc.value, t_decompress=td.value,
                compressed_bytes=cb.value, mismatches=mm.value)


def crc32_batch(data: np.ndarray, off: np.ndarray, ln: np.ndarray, kind: str = "port") -> np.ndarray:
    """enet_crc32 (packet.c:143-163) of every packet: the port's or the
    reference's own function (exported by libenet_ref.so)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(ln, dtype=np.uint32)
    out = np.zeros(len(ln), dtype=np.uint32)
    if kind == "port":
        lib = _load(PORT_SO)
        lib.or_crc32_batch.restype = None
        lib.or_crc32_batch(_ptr(data), _ptr(off), _ptr(ln), C.c_size_t(len(ln)), _ptr(out))
        return out
    lib = _load(REF_SO)
    lib.enet_crc32.restype = C.c_uint32
    lib.enet_crc32.argtypes = [C.c_void_p, C.c_size_t]
    base = data.ctypes.data
    buf = (_Buf * 1)()
    for i in range(len(ln)):
        buf[0].data = base + int(off[i])
        buf[0].dataLength = int(ln[i])
        out[i] = lib.enet_crc32(buf, 1)
    return out


# ----------------------------------------------------------- datagram framing
# Restatement of protocol.c's framing around the compressor and checksum
# callbacks -- test oracle for
# enet_rc_datagram_{encode,decode}_batch_*.
MTU = 4096                      # ENET_PROTOCOL_MAXIMUM_MTU (protocol.h:13) = sizeof packetData[1]


def _header_size(b0: int, checksum: bool) -> int:
    # protocol.c:1033-1035: 2 bytes, 4 with SENT_TIME (bit 15), + 4 for the checksum
    return (4 if b0 & 0x80 else 2) + (4 if checksum else 0)


def _crc(data: bytes, kind: str = "port") -> int:
    arr = np.frombuffer(bytes(data) + b"\0", np.uint8)
    return int(crc32_batch(arr, np.zeros(1, np.uint64), np.array([len(data)], np.uint32), kind)[0])


def datagram_encode(dgram: bytes, checksum: bool, seed: int, coder: "Coder") -> bytes:
    """protocol.c:1686-1718 for one assembled datagram (header, checksum field,
    uncompressed commands).  b"" for a datagram shorter than its header."""
    if len(dgram) < 2 or len(dgram) > MTU:
        return b""
    hs = _header_size(dgram[0], checksum)
    if len(dgram) < hs:
        return b""
    cmds = dgram[hs:]
    L = len(cmds)
    c, packed = coder.compress(cmds, out_limit=L, in_limit=L) if L else (0, b"")   # :1688-1694
    comp = 0 < c < L                                                                 # :1696
    b0 = (dgram[0] & ~0x40) | (0x40 if comp else 0)                                  # :1698, :1708
    head = bytes([b0]) + dgram[1:hs - (4 if checksum else 0)]
    if checksum:                                                                     # :1709-1718
        crc = _crc(head + int(seed).to_bytes(4, "little") + cmds)
        head += crc.to_bytes(4, "little")
    return head + (packed if comp else cmds)


def datagram_decode(wire: bytes, checksum: bool, seed: int, coder: "Coder") -> bytes:
    """protocol.c:1022-1091 for one received datagram: the bytes it goes on to
    parse (header + commands, checksum field = seed), or b"" where it drops it."""
    if len(wire) < 2:                                                                # :1022-1023
        return b""
    hs = _header_size(wire[0], checksum)
    if len(wire) < hs:
        return b""
    if wire[0] & 0x40:                                                               # :1052-1070
        r, data = coder.decompress(wire[hs:], MTU - hs)
        if r <= 0 or r > MTU - hs:
            return b""
        d = wire[:hs] + data
    else:
        if len(wire) > MTU:
            return b""
        d = bytes(wire)
    if checksum:                                                                     # :1072-1091
        want = int.from_bytes(d[hs - 4:hs], "little")
        d = d[:hs - 4] + int(seed).to_bytes(4, "little") + d[hs:]
        if _crc(d) != want:
            return b""
    return d
