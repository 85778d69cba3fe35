"""Multi-rank sharding of packet batches (enet_amd/shard.py) on CPU with gloo,
world_size 2 and 3: scatter from rank 0, per-rank coding, gather back, and the
reassembled result equals coding the whole batch on one rank.  The per-rank
coder here is the CPU oracle (test infrastructure); on GPUs the same code path
carries RCCL traffic between MI355X ranks."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from enet_amd import shard, synth  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.pyoracle import compress_batch
        if rank == 0:
            d, o, l = synth.mixed_batch(600, lo=1, hi=1500, seed=5)
            data, off, ln = torch.from_numpy(d), torch.from_numpy(o.astype(np.int64)), torch.from_numpy(l.astype(np.int32))
        else:
            data = off = ln = None
        pay, poff, pln = shard.scatter_batch(dist, data, off, ln)
        # code this rank's shard
        out, oo, cap, ol = compress_batch(pay.numpy(), poff.numpy().astype(np.uint64), pln.numpy().astype(np.uint32), "port")
        res, rl = shard.pack_results(torch.from_numpy(out), torch.from_numpy(oo.astype(np.int64)),
                                     torch.from_numpy(ol.astype(np.int32)))
        parts = shard.gather_results(dist, res, rl)
        if rank == 0:
            got = b"".join(bytes(p[0].numpy().tobytes()) for p in parts)
            got_len = np.concatenate([p[1].numpy() for p in parts])
            ref, roff, rcap, rlen = compress_batch(d, o, l, "port")
            want = b"".join(ref[int(roff[i]): int(roff[i]) + int(rlen[i])].tobytes() for i in range(len(rlen)))
            q.put((np.array_equal(got_len, rlen.astype(np.int32)), got == want, [int(p[1].numel()) for p in parts]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_scatter_code_gather_roundtrip(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    lens_ok, bytes_ok, counts = res
    assert lens_ok and bytes_ok
    assert sum(counts) == 600 and all(c > 0 for c in counts)


def test_shard_ranges_balance_bytes():
    l = synth.mixed_batch(10000)[2]
    rs = shard.shard_ranges(l, 8)
    assert rs[0][0] == 0 and rs[-1][1] == len(l)
    assert all(a <= b for a, b in rs) and all(rs[i][1] == rs[i + 1][0] for i in range(7))
    sums = [int(l[a:b].sum()) for a, b in rs]
    assert max(sums) - min(sums) <= 2 * int(l.max())
    assert shard.shard_ranges([5, 5], 4)[-1] == (2, 2)


def _worker_gpu(rank, world, port, q):
    """As _worker, but each rank codes its shard with the HIP coder on the
    box's one GPU (both directions, through shard.pack_results' device packing
    kernel); gloo carries the shards (host tensors)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from enet_amd import RangeCoder
        from oracle.pyoracle import compress_batch
        torch.cuda.set_device(0)
        if rank == 0:
            d, o, l = synth.mixed_batch(6000, lo=1, hi=1500, seed=6)
            data, off, ln = torch.from_numpy(d), torch.from_numpy(o.astype(np.int64)), torch.from_numpy(l.astype(np.int32))
        else:
            data = off = ln = None
        pay, poff, pln = shard.scatter_batch(dist, data, off, ln)
        rc = RangeCoder()
        dpay, doff, dln = pay.cuda(), poff.cuda(), pln.cuda()
        n = dln.numel()
        cap = (2 * dln.to(torch.int64) + 64).to(torch.int32)
        coff = torch.zeros(n, dtype=torch.int64, device="cuda")
        if n > 1:
            coff[1:] = torch.cumsum(cap[:-1].to(torch.int64), 0)
        cout = torch.zeros(int(coff[-1] + cap[-1]) if n else 1, dtype=torch.uint8, device="cuda")
        clen = torch.zeros(n, dtype=torch.int32, device="cuda")
        rc.compress_batch(dpay, doff, dln, cout, coff, cap, clen, max_len=int(dln.max().item()) if n else 16)
        back = torch.zeros_like(dpay)
        bl = torch.zeros(n, dtype=torch.int32, device="cuda")
        rc.decompress_batch(cout, coff, clen, back, doff, dln, bl, max_len=int(clen.max().item()) if n else 16)
        res, rl = shard.pack_results(cout, coff, clen, coder=rc)
        torch.cuda.synchronize()
        ok_local = bool(torch.equal(bl, dln)) and bool(torch.equal(back, dpay))
        parts = shard.gather_results(dist, res.cpu(), rl.cpu())
        okt = torch.tensor([1 if ok_local else 0])
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        rc.close()
        if rank == 0:
            got = b"".join(bytes(p[0].numpy().tobytes()) for p in parts)
            got_len = np.concatenate([p[1].numpy() for p in parts])
            ref, roff, rcap, rlen = compress_batch(d, o, l, "port")
            want = b"".join(ref[int(roff[i]): int(roff[i]) + int(rlen[i])].tobytes() for i in range(len(rlen)))
            q.put((np.array_equal(got_len, rlen.astype(np.int32)), got == want, bool(okt.item()),
                   [int(p[1].numel()) for p in parts]))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_scatter_code_gather_on_the_hip_coder():
    """shard.py's scatter / gather around the HIP coder (two ranks on the
    box's one GPU): each rank compresses and decompresses its shard on the
    GPU; the gathered compressed batch equals the oracle's, and every rank's
    round trip is exact."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_gpu, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    lens_ok, bytes_ok, rt_ok, counts = res
    assert lens_ok and bytes_ok and rt_ok
    assert sum(counts) == 6000 and all(c > 0 for c in counts)
