"""Sharding packet batches across GPUs.

Packets are independent (compress.c keeps no state across calls,
:252-265), so a batch shards into contiguous packet ranges with no exchange
during coding.  The only collectives are the scatter of a batch from a root
rank and the gather of the results, done with grouped point-to-point
send/recv -- on MI355X that is RCCL over the direct xGMI link between each
pair of GPUs (backend "nccl"); on CPU the same code runs over gloo, which is
how it is tested.

Layout on the wire, per destination rank: a small int64 header
[n_packets, payload_bytes], then the packet lengths (int32) and the payload
bytes (uint8); offsets are rebuilt locally as the exclusive cumsum of the
lengths.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


def shard_ranges(lengths: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous packet ranges [start, end) for ``world`` ranks with about
    equal payload bytes each (config C4 balances by sum of N)."""
    ln = np.asarray(lengths, dtype=np.int64)
    n = len(ln)
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    cum = np.concatenate([[0], np.cumsum(ln)])
    total = cum[-1]
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(cum, total * r / world, side="left")))
    cuts.append(n)
    cuts = np.maximum.accumulate(np.minimum(np.asarray(cuts), n))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def split_on_device(lengths, offsets, world: int):
    """shard_ranges computed where the batch lives (the GPU, on the GPU path),
    with the byte range of each part: ([(a, b)] * world, [(lo, hi)] * world).
    Only 3 world + 1 integers come back to the host -- not the lengths and
    offsets arrays.  The same split as enet_rc_multi_split / rc_multi_plan.hip:
    part k starts at the first packet whose exclusive prefix sum of lengths,
    times world, reaches total * k."""
    import torch
    n = lengths.numel()
    dev = lengths.device
    if world <= 1 or n == 0:
        hi = int((offsets[-1].to(torch.int64) + lengths[-1].to(torch.int64)).item()) if n else 0
        lo = int(offsets[0].item()) if n else 0
        return [(0, n)] + [(n, n)] * max(0, world - 1), [(lo, hi)] + [(0, 0)] * max(0, world - 1)
    ln = lengths.to(torch.int64)
    excl = torch.cumsum(ln, 0) - ln
    total = ln.sum()
    ks = torch.arange(1, world, dtype=torch.int64, device=dev)
    mid = torch.searchsorted(excl * world, total * ks)            # first index with excl * world >= total * k
    first = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), mid,
                       torch.full((1,), n, dtype=torch.int64, device=dev)])
    a, b = first[:-1], first[1:]
    last = torch.clamp(b - 1, min=0)
    off = offsets.to(torch.int64)
    lo = off[torch.clamp(a, max=n - 1)]
    hi = off[last] + ln[last]
    got = torch.cat([first, lo, hi]).cpu().tolist()               # the one read-back
    f, los, his = got[:world + 1], got[world + 1:2 * world + 1], got[2 * world + 1:]
    ranges = [(int(f[r]), int(f[r + 1])) for r in range(world)]
    spans = [(int(los[r]), int(his[r])) if f[r + 1] > f[r] else (0, 0) for r in range(world)]
    return ranges, spans


def _offsets(lengths):
    import torch
    off = torch.zeros_like(lengths, dtype=torch.int64)
    if lengths.numel() > 1:
        off[1:] = torch.cumsum(lengths[:-1].to(torch.int64), 0)
    return off


def _batch(dist, ops):
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()


def scatter_batch(dist, data, offsets, lengths, root: int = 0, device=None):
    """Scatter a packet batch held by ``root`` (``data``/``offsets``/``lengths``
    tensors; ignored on other ranks) into per-rank shards.  Every rank returns
    its shard as (data, offsets, lengths) on ``device``.

    Two grouped rounds: every rank's header at once, then every rank's
    lengths and payload at once -- the transfers to all ranks run together,
    one per xGMI link, instead of one rank after another."""
    import torch
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = device if device is not None else (data.device if data is not None else torch.device("cpu"))
    if rank == root:
        ranges, spans = split_on_device(lengths, offsets, world)
        hdrs, parts, keep = [], [], None
        for r, (a, b) in enumerate(ranges):
            lo, hi = spans[r]
            ln_r = lengths[a:b].to(device=dev, dtype=torch.int32).contiguous()
            pay = data[lo:hi].to(dev).contiguous()
            if r == root:
                keep = (pay, ln_r)
                continue
            hdrs.append(dist.P2POp(dist.isend, torch.tensor([b - a, hi - lo], dtype=torch.int64, device=dev), r))
            if b > a:
                parts += [dist.P2POp(dist.isend, ln_r, r), dist.P2POp(dist.isend, pay, r)]
        _batch(dist, hdrs)
        _batch(dist, parts)
        pay, ln_r = keep
        return pay, _offsets(ln_r), ln_r
    hdr = torch.zeros(2, dtype=torch.int64, device=dev)
    _batch(dist, [dist.P2POp(dist.irecv, hdr, root)])
    n, nbytes = int(hdr[0]), int(hdr[1])
    ln_r = torch.empty(n, dtype=torch.int32, device=dev)
    pay = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    if n:
        _batch(dist, [dist.P2POp(dist.irecv, ln_r, root), dist.P2POp(dist.irecv, pay, root)])
    return pay, _offsets(ln_r), ln_r


def pack_results(out, out_off, out_len, coder=None):
    """Compacts per-packet results (out[out_off[i] : +out_len[i]]) into one
    contiguous byte tensor; returns (bytes, lengths).  Device tensors go
    through the library's packing kernel (rc_pack.hip,
    enet_rc_pack_batch_device: one wavefront per packet, no per-byte index);
    host tensors (the CPU tests) are sliced on the host."""
    import torch
    n = out_len.numel()
    if n == 0:
        return torch.empty(0, dtype=torch.uint8, device=out.device), out_len
    ln = out_len.to(torch.int64)
    total = int(ln.sum().item())
    packed = torch.empty(max(total, 1), dtype=torch.uint8, device=out.device)
    if out.is_cuda:
        if coder is None:
            raise ValueError("pack_results on device tensors needs a RangeCoder (the packing kernel)")
        oo = out_off.to(torch.int64).contiguous()
        ol = out_len.to(torch.int32).contiguous()
        stream = torch.cuda.current_stream(out.device)
        rc = coder.lib.enet_rc_pack_batch_device(coder.ctx, out.data_ptr(), oo.data_ptr(), ol.data_ptr(), n,
                                                 packed.data_ptr(), stream.cuda_stream)
        if rc != 0:
            raise RuntimeError(f"enet_rc_pack_batch_device failed: HIP error {rc}")
        return packed[:total], out_len
    o, l = out_off.numpy(), out_len.numpy()
    src = out.numpy()
    if total:
        packed.numpy()[:total] = np.concatenate([src[int(o[i]): int(o[i]) + int(l[i])] for i in range(n)])
    return packed[:total], out_len


def gather_results(dist, payload, lengths, root: int = 0):
    """Gather each rank's packed results (bytes + int32 lengths) to ``root``.
    Returns on root a list of (payload, lengths) in rank order; None elsewhere.
    Two grouped rounds as in scatter_batch: all headers, then all payloads."""
    import torch
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = payload.device
    if rank != root:
        hdr = torch.tensor([lengths.numel(), payload.numel()], dtype=torch.int64, device=dev)
        _batch(dist, [dist.P2POp(dist.isend, hdr, root)])
        if lengths.numel():
            _batch(dist, [dist.P2POp(dist.isend, lengths.to(torch.int32).contiguous(), root),
                          dist.P2POp(dist.isend, payload.contiguous(), root)])
        return None
    hdrs = {r: torch.zeros(2, dtype=torch.int64, device=dev) for r in range(world) if r != root}
    _batch(dist, [dist.P2POp(dist.irecv, h, r) for r, h in hdrs.items()])
    parts = [None] * world
    parts[root] = (payload, lengths)
    ops = []
    for r, h in hdrs.items():
        n, nb = int(h[0]), int(h[1])
        ln = torch.empty(n, dtype=torch.int32, device=dev)
        pay = torch.empty(nb, dtype=torch.uint8, device=dev)
        if n:
            ops += [dist.P2POp(dist.irecv, ln, r), dist.P2POp(dist.irecv, pay, r)]
        parts[r] = (pay, ln)
    _batch(dist, ops)
    return parts
