"""One process, several GPUs through the C ABI (enet_rc_multi_*, rc_multi.c;
SURVEY.md §8e).  CPU: the split against enet_amd/shard.py's ranges.  GPU:
bit-exact results against the oracle with the device lists [0] (one device),
[0, 0, 0] (three contexts on the one GPU of the test box: the non-root ranges
take the whole scatter / code / gather path of a multi-GPU node, over a
same-device "peer" copy and the root's direct read of the device's slots) and
[0, 0] with a batch whose second range is empty.  Multi-GPU scaling itself is
unmeasured here (one GPU per test box)."""
import numpy as np
import pytest

from enet_amd import multi_plan, multi_split, shard, synth


@pytest.mark.parametrize("n,parts", [(0, 3), (1, 4), (7, 8), (1000, 1), (1000, 3), (65536, 8), (100000, 5)])
def test_split_matches_shard_ranges(n, parts):
    rng = np.random.default_rng(n + parts)
    ln = rng.integers(0, 1400, size=n).astype(np.uint32)
    first = multi_split(ln, parts)
    want = shard.shard_ranges(ln, parts)
    assert [int(x) for x in first[:-1]] == [a for a, _ in want]
    assert int(first[-1]) == n
    assert all(first[k] <= first[k + 1] for k in range(parts))
    if n and ln.sum():
        per = [int(ln[int(first[k]): int(first[k + 1])].sum()) for k in range(parts)]
        assert max(per) - min(per) <= 2 * 1400         # balanced by payload bytes within a packet or two


def test_split_bad_arguments():
    with pytest.raises(ValueError):
        multi_split(np.zeros(4, np.uint32), 0)
    with pytest.raises(ValueError):
        multi_split(np.zeros(4, np.uint32), 65)


def _plan_case(n, seed):
    """ragged lengths (zeros included), offsets in no particular order, caps 2N + 64"""
    rng = np.random.default_rng(seed)
    ln = rng.integers(0, 1400, size=n).astype(np.uint32)
    ln[rng.random(n) < 0.05] = 0
    ioff = rng.permutation(np.arange(n, dtype=np.uint64) * 1500) + 3
    cap = (2 * ln.astype(np.uint64) + 64).astype(np.uint32)
    ooff = rng.permutation(np.arange(n, dtype=np.uint64) * 3000)
    return ln, ioff, ooff, cap


def _plan_numpy(ln, ioff, ooff, cap, parts):
    first = multi_split(ln, parts)
    ext = []
    for k in range(parts):
        a, b = int(first[k]), int(first[k + 1])
        if a == b:
            ext += [2 ** 64 - 1, 0, 2 ** 64 - 1, 0]
        else:
            ext += [int(ioff[a:b].min()), int((ioff[a:b] + ln[a:b]).max()),
                    int(ooff[a:b].min()), int((ooff[a:b] + cap[a:b]).max())]
    return [int(x) for x in first] + ext


@pytest.mark.parametrize("n,parts", [(1, 1), (1, 5), (7, 8), (1000, 3), (5000, 64), (70000, 8)])
def test_plan_host_mirror(n, parts):
    """enet_rc_multi_plan (the host restatement of rc_multi_plan.hip) against numpy"""
    ln, ioff, ooff, cap = _plan_case(n, n + parts)
    assert [int(x) for x in multi_plan(ln, ioff, ooff, cap, parts)] == _plan_numpy(ln, ioff, ooff, cap, parts)
    z = np.zeros(n, np.uint32)           # no payload: every split point 0
    got = multi_plan(z, ioff, ooff, cap, parts)
    assert [int(x) for x in got[:parts]] == [0] * parts and int(got[parts]) == n


@pytest.mark.parametrize("n,parts", [(0, 2), (1, 1), (1, 5), (7, 8), (1000, 3), (5000, 64), (70000, 8)])
def test_shard_split_on_device_mirror(n, parts):
    """shard.split_on_device (the split shard.scatter_batch computes where the
    batch lives, CPU tensors here) against shard_ranges and the C split, with
    unequal lengths, zero-length packets, and parts left empty"""
    torch = pytest.importorskip("torch")
    ln, ioff, ooff, cap = _plan_case(n, n * 5 + parts)
    for lens in (ln, np.zeros(n, np.uint32), np.where(np.arange(n) == n - 1, 1000, 0).astype(np.uint32)):
        off = np.zeros(n, np.int64)
        if n > 1:
            off[1:] = np.cumsum(lens[:-1].astype(np.int64))
        ranges, spans = shard.split_on_device(torch.from_numpy(lens.astype(np.int32)), torch.from_numpy(off), parts)
        assert ranges == shard.shard_ranges(lens, parts)
        if n:
            assert [a for a, _ in ranges] + [n] == [int(x) for x in multi_split(lens, parts)]
        for (a, b), (lo, hi) in zip(ranges, spans):
            if a < b:
                assert (lo, hi) == (int(off[a]), int(off[b - 1] + lens[b - 1]))
            else:
                assert (lo, hi) == (0, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("n,parts", [(1, 1), (1, 5), (7, 8), (1000, 3), (5000, 64), (70000, 8), (300000, 3)])
def test_plan_device_matches_host(n, parts):
    """rc_multi_plan.hip (the split rc_multi.c computes on the root) against its host restatement"""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ln, ioff, ooff, cap = _plan_case(n, n * 3 + parts)
    for lens in (ln, np.zeros(n, np.uint32)):
        dev = [torch.from_numpy(a.astype(t)).cuda() for a, t in
               ((lens, np.int32), (ioff, np.int64), (ooff, np.int64), (cap, np.int32))]
        got = multi_plan(*dev, parts, device=True)
        assert np.array_equal(got, multi_plan(lens, ioff, ooff, cap, parts)), (n, parts)


def _oracle(d, o, l):
    from oracle.pyoracle import compress_batch as ocompress
    return ocompress(d, o, l, "port")


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
def test_multi_host_batches_vs_oracle(devices):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from enet_amd import MultiCoder
    from oracle.pyoracle import fnv_digest
    d, o, l = synth.mixed_batch(20000, seed=0x4D554C54)
    want, wo, wcap, wl = _oracle(d, o, l)
    n = len(l)
    ln = l.astype(np.uint32)
    cap = (2 * ln.astype(np.int64) + 64).astype(np.uint32)
    coff = np.zeros(n, np.uint64)
    coff[1:] = np.cumsum(cap[:-1].astype(np.uint64) + 5)          # gapped slots
    cout = np.zeros(int(coff[-1] + cap[-1]) + 16, np.uint8)
    clen = np.zeros(n, np.uint32)
    m = MultiCoder(devices)
    m.batch_host(False, d, o, ln, cout, coff, cap, clen)
    assert np.array_equal(clen, wl)
    assert fnv_digest(cout, coff, clen) == fnv_digest(want, wo, wl)
    dout = np.zeros(d.size + 16, np.uint8)
    dlen = np.zeros(n, np.uint32)
    m.batch_host(True, cout, coff, clen, dout, o, ln, dlen)
    assert np.array_equal(dlen, ln)
    assert np.array_equal(dout[: d.size], d)
    m.close()


@pytest.mark.gpu
@pytest.mark.parametrize("devices,stage", [([0], False), ([0, 0, 0], False), ([0, 0, 0], True)])
def test_multi_device_batches_vs_oracle(devices, stage, monkeypatch):
    """stage: ENET_RC_MULTI_NO_PEER=1, the non-root ranges' results through the
    root's stage buffer (rc_multi.c: the path of distinct devices) on the one
    GPU of the test box; the gaps between slots stay untouched either way."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if stage:
        monkeypatch.setenv("ENET_RC_MULTI_NO_PEER", "1")
    from enet_amd import MultiCoder
    from oracle.pyoracle import fnv_digest
    d, o, l = synth.mixed_batch(20000, seed=0x4D554C55)
    want, wo, wcap, wl = _oracle(d, o, l)
    n = len(l)
    dev = lambda a, t: torch.from_numpy(np.ascontiguousarray(a)).to(t).cuda()  # noqa: E731
    din, doff, dlen = dev(d, torch.uint8), dev(o, torch.int64), dev(l, torch.int32)
    cap = (2 * dlen.to(torch.int64) + 64).to(torch.int32)
    gap = 7
    coff = torch.zeros(n, dtype=torch.int64, device="cuda")
    coff[1:] = torch.cumsum(cap[:-1].to(torch.int64) + gap, 0)
    total = int(coff[-1] + cap[-1]) + gap
    cout = torch.full((total,), 0xA5, dtype=torch.uint8, device="cuda")
    clen = torch.zeros(n, dtype=torch.int32, device="cuda")
    m = MultiCoder(devices)
    m.batch_device(False, din, doff, dlen, cout, coff, cap, clen, max_len=int(l.max()))
    cl = clen.cpu().numpy().astype(np.uint32)
    assert np.array_equal(cl, wl)
    cb, co = cout.cpu().numpy(), coff.cpu().numpy().astype(np.uint64)
    assert fnv_digest(cb, co, cl) == fnv_digest(want, wo, wl)
    # nothing written outside [out_off, out_off + out_len)
    mask = np.ones(total, bool)
    for i in range(n):
        mask[int(co[i]): int(co[i]) + int(cl[i])] = False
    assert (cb[mask] == 0xA5).all()
    dout = torch.zeros_like(din)
    dl = torch.zeros(n, dtype=torch.int32, device="cuda")
    # decompress into gapped slots over a canary: nothing written past out_len
    dcap = dlen + 5
    doff2 = torch.zeros(n, dtype=torch.int64, device="cuda")
    doff2[1:] = torch.cumsum(dcap[:-1].to(torch.int64) + gap, 0)
    dtot = int(doff2[-1] + dcap[-1]) + gap
    dout = torch.full((dtot,), 0x5A, dtype=torch.uint8, device="cuda")
    dl = torch.zeros(n, dtype=torch.int32, device="cuda")
    m.batch_device(True, cout, coff, clen, dout, doff2, dcap, dl, max_len=int(cl.max()))
    assert torch.equal(dl, dlen)
    db, do2 = dout.cpu().numpy(), doff2.cpu().numpy()
    dmask = np.ones(dtot, bool)
    for i in range(n):
        a = int(do2[i])
        assert np.array_equal(db[a: a + int(l[i])], d[int(o[i]): int(o[i]) + int(l[i])]), i
        dmask[a: a + int(l[i])] = False
    assert (db[dmask] == 0x5A).all()
    m.close()


@pytest.mark.gpu
def test_multi_device_empty_range_and_stream():
    """[0, 0] with every payload byte in the last packet: the second device's
    range is empty (the plan's split puts all packets on the root).  Then a
    batch whose inputs are written on a side stream: the root waits for that
    stream (the _stream entry), not for the null stream."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from enet_amd import MultiCoder
    from oracle.pyoracle import compress_batch as ocompress, fnv_digest
    n = 3000
    rng = np.random.default_rng(77)
    ln = np.zeros(n, np.uint32)
    ln[-1] = 1200
    d = rng.integers(0, 256, size=1200, dtype=np.uint8)
    o = np.full(n, 0, np.uint64)
    first = multi_split(ln, 2)
    assert int(first[1]) == n - 1 or int(first[1]) == n          # one part holds every packet with payload
    dev = lambda a, t: torch.from_numpy(np.ascontiguousarray(a)).to(t).cuda()  # noqa: E731
    m = MultiCoder([0, 0])
    for side in (False, True):
        s = torch.cuda.Stream() if side else torch.cuda.current_stream()
        with torch.cuda.stream(s):
            din, doff, dlen = dev(d, torch.uint8), dev(o, torch.int64), dev(ln, torch.int32)
            cap = (2 * dlen.to(torch.int64) + 64).to(torch.int32)
            coff = torch.zeros(n, dtype=torch.int64, device="cuda")
            coff[1:] = torch.cumsum(cap[:-1].to(torch.int64), 0)
            cout = torch.zeros(int(coff[-1] + cap[-1]), dtype=torch.uint8, device="cuda")
            clen = torch.full((n,), 77, dtype=torch.int32, device="cuda")
            m.batch_device(False, din, doff, dlen, cout, coff, cap, clen, max_len=1200)
        torch.cuda.synchronize()
        want, wo, wcap, wl = ocompress(d, o, ln, "port")
        cl = clen.cpu().numpy().astype(np.uint32)
        assert np.array_equal(cl, wl)
        assert fnv_digest(cout.cpu().numpy(), coff.cpu().numpy().astype(np.uint64), cl) == fnv_digest(want, wo, wl)
    m.close()
