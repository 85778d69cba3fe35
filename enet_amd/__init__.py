"""enet_amd -- MI355X-native drop-in for ENet's range-coder packet compressor.

The product is ``enet_amd/lib/libenet_rc_amd.so`` (C host shim + gfx950 HIP
kernels, C ABI in ``include/enet_rc_amd.h``).  This Python package is a thin
ctypes front end used by the tests and the benchmark:

* :class:`RangeCoder` mirrors the reference's ``ENetCompressor`` plugin
  (``enet_range_coder_create/compress/decompress/destroy``, enet.h:603-606):
  same arguments, same ``0``-on-failure convention.
* :func:`compress_batch` / :func:`decompress_batch` run whole packet batches
  resident in device memory (torch tensors on ``cuda``), one wavefront per
  packet.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

from ._lib import ENetBuffer, get_lib

__all__ = ["RangeCoder", "MultiCoder", "compress_batch", "decompress_batch", "get_lib", "ENetBuffer",
           "multi_split", "multi_plan"]


class RangeCoder:
    """One coder context: ``enet_range_coder_create`` (compress.c:48-56)."""

    def __init__(self):
        self.lib = lib = get_lib()
        self.ctx = lib.enet_range_coder_create()
        if not self.ctx:
            raise RuntimeError("enet_range_coder_create failed (no usable HIP device?)")

    def close(self):
        if self.ctx:
            self.lib.enet_range_coder_destroy(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- reference per-datagram surface (compress.c:246, :498) ---------------
    def compress_gather(self, backing: bytes, spans: Sequence[tuple], in_limit: int, out_limit: int):
        """Gather-list compress; ``spans`` = [(start, length)] into ``backing``.
        Returns ``(return_value, bytes)`` like the reference call."""
        buf = C.create_string_buffer(bytes(backing) + b"\0" * 8)
        base = C.addressof(buf)
        arr = (ENetBuffer * max(1, len(spans)))()
        for i, (s, l) in enumerate(spans):
            arr[i].data = base + s
            arr[i].dataLength = l
        out = C.create_string_buffer(max(1, out_limit))
        r = self.lib.enet_range_coder_compress(self.ctx, arr, len(spans), in_limit, C.addressof(out), out_limit)
        return int(r), out.raw[: r]

    def compress_gather_batch(self, backing: bytes, lists: Sequence[Sequence[tuple]], out_caps: Sequence[int]):
        """Batch of gather lists (``enet_rc_compress_gather_batch_host``):
        packet i is the spans ``lists[i]`` = [(start, length)] into
        ``backing``, consumed like ``compress_gather``.  Returns a list of
        ``(return_value, bytes)``."""
        import numpy as np
        buf = C.create_string_buffer(bytes(backing) + b"\0" * 8)
        base = C.addressof(buf)
        nb = sum(len(l) for l in lists)
        arr = (ENetBuffer * max(1, nb))()
        first = np.zeros(len(lists) + 1, dtype=np.uint64)
        k = 0
        for i, spans in enumerate(lists):
            first[i] = k
            for s, l in spans:
                arr[k].data = base + s
                arr[k].dataLength = l
                k += 1
        first[len(lists)] = k
        caps = np.asarray(out_caps, dtype=np.uint32)
        offs = np.zeros(len(lists), dtype=np.uint64)
        if len(lists) > 1:
            offs[1:] = np.cumsum(caps[:-1], dtype=np.uint64)
        out = np.zeros(int(caps.sum()) + 1, dtype=np.uint8)
        olen = np.zeros(len(lists), dtype=np.uint32)
        rc = self.lib.enet_rc_compress_gather_batch_host(self.ctx, arr, first.ctypes.data, len(lists), out.ctypes.data,
                                                         offs.ctypes.data, caps.ctypes.data, olen.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"enet_rc_compress_gather_batch_host failed: HIP error {rc}")
        return [(int(olen[i]), out[int(offs[i]): int(offs[i]) + int(olen[i])].tobytes()) for i in range(len(lists))]

    def compress(self, data: bytes, out_limit: Optional[int] = None, in_limit: Optional[int] = None):
        if out_limit is None:
            out_limit = 2 * len(data) + 64
        if in_limit is None:
            in_limit = len(data)
        return self.compress_gather(data, [(0, len(data))], in_limit, out_limit)

    def decompress(self, data: bytes, out_limit: int = 4096):
        src = C.create_string_buffer(bytes(data) + b"\0")
        out = C.create_string_buffer(max(1, out_limit))
        r = self.lib.enet_range_coder_decompress(self.ctx, C.addressof(src), len(data), C.addressof(out), out_limit)
        return int(r), out.raw[: r]

    # -- batch surface ---------------------------------------------------------
    def _batch(self, fn, inp, in_off, in_len, max_len, out, out_off, out_cap, out_len, stream):
        import torch
        for t in (inp, in_off, in_len, out, out_off, out_cap, out_len):
            if not (t.is_cuda and t.is_contiguous()):
                raise ValueError("batch tensors must be contiguous device tensors")
        assert inp.dtype == torch.uint8 and out.dtype == torch.uint8
        assert in_off.dtype == torch.int64 and out_off.dtype == torch.int64
        assert in_len.dtype == torch.int32 and out_cap.dtype == torch.int32 and out_len.dtype == torch.int32
        n = in_len.numel()
        if stream is None:
            stream = torch.cuda.current_stream(inp.device)
        rc = fn(self.ctx, inp.data_ptr(), in_off.data_ptr(), in_len.data_ptr(), n, int(max_len),
                out.data_ptr(), out_off.data_ptr(), out_cap.data_ptr(), out_len.data_ptr(),
                C.c_void_p(stream.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"enet_rc batch failed: HIP error {rc}")

    def compress_batch(self, inp, in_off, in_len, out, out_off, out_cap, out_len, max_len=0, stream=None):
        self._batch(self.lib.enet_rc_compress_batch_device, inp, in_off, in_len, max_len, out, out_off,
                    out_cap, out_len, stream)

    def decompress_batch(self, inp, in_off, in_len, out, out_off, out_cap, out_len, max_len=0, stream=None,
                         max_out=0):
        """max_out: an upper bound of out_cap[] (0 = unknown); with it, small
        batches decode with a right-sized model (enet_rc_decompress_batch_device_bounded)."""
        if max_out:
            fn = self.lib.enet_rc_decompress_batch_device_bounded
            self._batch(lambda *a: fn(*a[:-1], max_out, a[-1]), inp, in_off, in_len, max_len, out, out_off,
                        out_cap, out_len, stream)
            return
        self._batch(self.lib.enet_rc_decompress_batch_device, inp, in_off, in_len, max_len, out, out_off,
                    out_cap, out_len, stream)

    def crc32_batch(self, inp, in_off, in_len, crc_out=None, stream=None):
        """enet_crc32 (packet.c:143-163) of every packet, on the GPU.  Returns an
        int32 device tensor holding the reference's uint32 results (network
        byte order, as written into ENet datagram headers)."""
        import torch
        for t in (inp, in_off, in_len):
            if not (t.is_cuda and t.is_contiguous()):
                raise ValueError("batch tensors must be contiguous device tensors")
        assert inp.dtype == torch.uint8 and in_off.dtype == torch.int64 and in_len.dtype == torch.int32
        n = in_len.numel()
        if crc_out is None:
            crc_out = torch.empty(n, dtype=torch.int32, device=inp.device)
        assert crc_out.is_cuda and crc_out.dtype == torch.int32 and crc_out.numel() >= n
        if stream is None:
            stream = torch.cuda.current_stream(inp.device)
        rc = self.lib.enet_rc_crc32_batch_device(self.ctx, inp.data_ptr(), in_off.data_ptr(), in_len.data_ptr(),
                                                 n, crc_out.data_ptr(), C.c_void_p(stream.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"enet_rc_crc32_batch_device failed: HIP error {rc}")
        return crc_out

    def crc32(self, data: bytes) -> int:
        """One datagram through the host-pointer batch path (like enet_crc32 on one buffer)."""
        src = C.create_string_buffer(bytes(data) + b"\0")
        off = (C.c_uint64 * 1)(0)
        ln = (C.c_uint32 * 1)(len(data))
        out = (C.c_uint32 * 1)(0)
        rc = self.lib.enet_rc_crc32_batch_host(self.ctx, C.addressof(src), off, ln, 1, out)
        if rc != 0:
            raise RuntimeError(f"enet_rc_crc32_batch_host failed: HIP error {rc}")
        return int(out[0])

    def _dgram(self, fn, inp, in_off, in_len, out, out_off, out_len, checksum, seed, stream):
        import torch
        for t in (inp, in_off, in_len, out, out_off, out_len):
            if not (t.is_cuda and t.is_contiguous()):
                raise ValueError("datagram tensors must be contiguous device tensors")
        assert inp.dtype == torch.uint8 and out.dtype == torch.uint8
        assert in_off.dtype == torch.int64 and out_off.dtype == torch.int64
        assert in_len.dtype == torch.int32 and out_len.dtype == torch.int32
        n = in_len.numel()
        if checksum:
            assert seed is not None and seed.is_cuda and seed.dtype == torch.int32 and seed.numel() >= n
        if stream is None:
            stream = torch.cuda.current_stream(inp.device)
        rc = fn(self.ctx, inp.data_ptr(), in_off.data_ptr(), in_len.data_ptr(), n, 1 if checksum else 0,
                seed.data_ptr() if checksum else None, out.data_ptr(), out_off.data_ptr(), out_len.data_ptr(),
                C.c_void_p(stream.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"enet_rc datagram batch failed: HIP error {rc}")

    def datagram_encode_batch(self, inp, in_off, in_len, out, out_off, out_len, checksum=False, seed=None,
                              stream=None):
        """protocol.c:1686-1718 for n assembled datagrams (device tensors): wire
        datagrams into out at out_off (slot >= in_len), lengths into out_len.
        seed: int32 tensor of connectIDs (or 0) when checksum."""
        self._dgram(self.lib.enet_rc_datagram_encode_batch_device, inp, in_off, in_len, out, out_off, out_len,
                    checksum, seed, stream)

    def datagram_decode_batch(self, inp, in_off, in_len, out, out_off, out_len, checksum=False, seed=None,
                              stream=None):
        """protocol.c:1022-1091 for n received datagrams (device tensors): 4096-B
        slots of out at out_off get header + commands; out_len 0 = dropped."""
        self._dgram(self.lib.enet_rc_datagram_decode_batch_device, inp, in_off, in_len, out, out_off, out_len,
                    checksum, seed, stream)

    def datagrams(self, decode: bool, datagrams, checksum=False, seeds=None):
        """Host-memory convenience over the *_batch_host calls: list of bytes in,
        list of bytes out (b"" where protocol.c drops the datagram)."""
        import numpy as np
        n = len(datagrams)
        if n == 0:
            return []
        ln = np.array([len(d) for d in datagrams], np.uint32)
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
        blob = np.frombuffer(b"".join(datagrams) + b"\0" * 16, np.uint8).copy()
        slot = 4096 if decode else int(max(ln.max(), 1))
        out_off = (np.arange(n, dtype=np.uint64) * np.uint64(slot))
        out = np.zeros(n * slot + 16, np.uint8)
        out_len = np.zeros(n, np.uint32)
        sd = np.asarray(seeds if seeds is not None else np.zeros(n), dtype=np.uint32)
        p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
        fn = self.lib.enet_rc_datagram_decode_batch_host if decode else self.lib.enet_rc_datagram_encode_batch_host
        rc = fn(self.ctx, p(blob), p(off), p(ln), n, 1 if checksum else 0, p(sd), p(out), p(out_off), p(out_len))
        if rc != 0:
            raise RuntimeError(f"enet_rc datagram host batch failed: HIP error {rc}")
        return [out[int(out_off[i]): int(out_off[i]) + int(out_len[i])].tobytes() for i in range(n)]

    def last_exact_count(self) -> int:
        return int(self.lib.enet_rc_last_exact_count(self.ctx))

    def last_lane_count(self) -> int:
        """Packets of the last batch the first pass (two-pass encoder or
        bucket-history decoder) left to the lane kernels."""
        return int(self.lib.enet_rc_last_lane_count(self.ctx))


def multi_split(in_len, parts: int):
    """enet_rc_multi_split: device k codes packets [first[k], first[k+1])."""
    import numpy as np
    ln = np.ascontiguousarray(in_len, dtype=np.uint32)
    first = np.zeros(parts + 1, np.uint64)
    rc = get_lib().enet_rc_multi_split(ln.ctypes.data, len(ln), parts, first.ctypes.data)
    if rc != 0:
        raise ValueError("enet_rc_multi_split: bad arguments")
    return first


def multi_plan(in_len, in_off, out_off, out_cap, parts: int, device: bool = False):
    """enet_rc_multi_plan (host arrays) or, device=True, enet_rc_multi_plan_device
    (CUDA tensors: uint32/int32 lengths and caps, int64 offsets): first[0..parts]
    and each part's (lowest in_off, highest in_off + in_len, lowest out_off,
    highest out_off + out_cap), as an array of 5 parts + 1 uint64 words."""
    import numpy as np
    plan = np.zeros(5 * parts + 1, np.uint64)
    lib = get_lib()
    if device:
        n = in_len.numel()
        rc = lib.enet_rc_multi_plan_device(in_len.data_ptr(), in_off.data_ptr(), out_off.data_ptr(),
                                           out_cap.data_ptr(), n, parts, plan.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"enet_rc_multi_plan_device failed: HIP error {rc}")
        return plan
    arrs = [np.ascontiguousarray(a, dtype=t) for a, t in
            ((in_len, np.uint32), (in_off, np.uint64), (out_off, np.uint64), (out_cap, np.uint32))]
    rc = lib.enet_rc_multi_plan(arrs[0].ctypes.data, arrs[1].ctypes.data, arrs[2].ctypes.data, arrs[3].ctypes.data,
                                len(arrs[0]), parts, plan.ctypes.data)
    if rc != 0:
        raise ValueError("enet_rc_multi_plan: bad arguments")
    return plan


class MultiCoder:
    """One process, several GPUs (enet_rc_multi_*, rc_multi.c): a context per
    listed device; batches split by payload bytes across them."""

    def __init__(self, devices: Sequence[int]):
        self.lib = lib = get_lib()
        arr = (C.c_int * len(devices))(*devices)
        self.ctx = lib.enet_rc_multi_create(arr, len(devices))
        if not self.ctx:
            raise RuntimeError(f"enet_rc_multi_create({list(devices)}) failed")

    def close(self):
        if self.ctx:
            self.lib.enet_rc_multi_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def batch_host(self, decompress: bool, data, off, ln, out, out_off, out_cap, out_len):
        """numpy arrays (uint8, uint64, uint32, uint8, uint64, uint32, uint32)."""
        fn = self.lib.enet_rc_multi_decompress_batch_host if decompress else self.lib.enet_rc_multi_compress_batch_host
        p = lambda a: a.ctypes.data  # noqa: E731
        rc = fn(self.ctx, p(data), p(off), p(ln), len(ln), p(out), p(out_off), p(out_cap), p(out_len))
        if rc != 0:
            raise RuntimeError(f"enet_rc_multi host batch failed: HIP error {rc}")

    def batch_device(self, decompress: bool, inp, in_off, in_len, out, out_off, out_cap, out_len, max_len=0,
                     stream=None):
        """torch tensors on the first listed device (the batch's dtypes as RangeCoder.compress_batch).
        The inputs are taken in the order of `stream` (default: torch's current stream on that
        device), which the root device's work waits for on the GPU."""
        import torch
        fn = self.lib.enet_rc_multi_decompress_batch_device_stream if decompress else \
            self.lib.enet_rc_multi_compress_batch_device_stream
        st = stream if stream is not None else torch.cuda.current_stream(inp.device)
        rc = fn(self.ctx, inp.data_ptr(), in_off.data_ptr(), in_len.data_ptr(), in_len.numel(), int(max_len),
                out.data_ptr(), out_off.data_ptr(), out_cap.data_ptr(), out_len.data_ptr(), st.cuda_stream)
        if rc != 0:
            raise RuntimeError(f"enet_rc_multi device batch failed: HIP error {rc}")


def _caps_offsets(caps):
    import torch
    off = torch.zeros_like(caps, dtype=torch.int64)
    if caps.numel() > 1:
        off[1:] = torch.cumsum(caps[:-1].to(torch.int64), 0)
    return off


def compress_batch(coder: RangeCoder, inp, in_off, in_len, max_len: int, out_cap=None):
    """Allocates outputs (default capacity 2N+64 per packet) and compresses.
    Returns ``(out, out_off, out_cap, out_len)`` device tensors."""
    import torch
    if out_cap is None:
        out_cap = (2 * in_len.to(torch.int64) + 64).to(torch.int32)
    out_off = _caps_offsets(out_cap)
    total = int(out_off[-1].item() + out_cap[-1].item()) if out_cap.numel() else 0
    out = torch.empty(max(total, 1), dtype=torch.uint8, device=inp.device)
    out_len = torch.empty_like(in_len)
    coder.compress_batch(inp, in_off, in_len, out, out_off, out_cap, out_len, max_len)
    return out, out_off, out_cap, out_len


def decompress_batch(coder: RangeCoder, inp, in_off, in_len, out_cap, max_len: int = 0,
                     max_out: Optional[int] = None):
    """Allocates outputs of out_cap[i] bytes per packet and decompresses.
    ``max_out`` bounds out_cap[] (default: its maximum), so small batches get
    the right-sized decoder (enet_rc_decompress_batch_device_bounded).
    Returns ``(out, out_off, out_len)`` device tensors."""
    import torch
    out_off = _caps_offsets(out_cap)
    total = int(out_off[-1].item() + out_cap[-1].item()) if out_cap.numel() else 0
    out = torch.empty(max(total, 1), dtype=torch.uint8, device=inp.device)
    out_len = torch.empty_like(in_len)
    if max_out is None:
        max_out = max(int(out_cap.max().item()), 0) if out_cap.numel() else 0
    coder.decompress_batch(inp, in_off, in_len, out, out_off, out_cap, out_len, max_len, max_out=max_out)
    return out, out_off, out_len
