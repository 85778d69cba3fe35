"""Host-pointer batches and the caller's memory (rc_host.c run_host /
host_results), against the oracle:

- the GPU gather of a gapped compressed input over the caller's mapped,
  page-locked range (rc_gather16 over a buffer the caller page-locked) when
  the CPU rewrites that buffer between calls, and when the buffer is freed
  and a new one takes its place -- the round-5 review's candidate (b) for the
  r5a wrong decode (stale lines of mapped pages); the same batches from
  pageable memory take the pinned staging (pageable caller memory is not
  page-locked per call unless ENET_RC_HOST_REGISTER=1);
- back-to-back output slots that some packets do not fill (corrupt streams):
  the caller's bytes past each out_len stay as they were, as compress.c
  writes only what it decodes (round-5 ADVICE: the one-DMA result path).
"""
import ctypes as C

import numpy as np
import pytest

from enet_amd import synth

pytestmark = pytest.mark.gpu

P = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731


@pytest.fixture(scope="module")
def rc():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from enet_amd import RangeCoder
    c = RangeCoder()
    yield c
    c.close()


def _pinned(nbytes, fill=None):
    import torch
    a = torch.empty(nbytes, dtype=torch.uint8).pin_memory().numpy()
    if fill is not None:
        a[:] = fill
    return a


def _oracle_streams(d, o, l):
    from oracle.pyoracle import compress_batch
    out, oo, cap, ol = compress_batch(d, o, l, "port")
    return [out[int(oo[i]): int(oo[i]) + int(ol[i])] for i in range(len(l))]


@pytest.mark.parametrize("mem", ["pinned", "pageable"])
def test_zero_copy_input_rewritten_between_calls(rc, mem):
    n = 30000
    a = synth.mixed_batch(n, seed=0x5A31)
    b = synth.mixed_batch(n, seed=0x5A32)
    sa, sb = _oracle_streams(*a), _oracle_streams(*b)
    # gapped slots, not at a uniform pitch: the GPU gather over the mapped caller range
    cap = np.array([max(len(x), len(y)) + 16 + (i % 7) for i, (x, y) in enumerate(zip(sa, sb))], np.uint64)
    coff = np.zeros(n, np.uint64)
    coff[1:] = np.cumsum(cap[:-1])
    total = int(coff[-1] + cap[-1])

    def fill(buf, which):
        lens = np.zeros(n, np.uint32)
        for i in range(n):
            s = (sa if which[i] == 0 else sb)[i]
            buf[int(coff[i]): int(coff[i]) + len(s)] = s
            lens[i] = len(s)
        return lens

    def check(buf, lens, which):
        dout = np.zeros(int(a[2].sum()) + int(b[2].sum()) + 64, np.uint8)
        ln = np.where(which == 0, a[2], b[2]).astype(np.uint32)
        oo = np.zeros(n, np.uint64)
        oo[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
        got = np.zeros(n, np.uint32)
        assert rc.lib.enet_rc_decompress_batch_host(rc.ctx, P(buf), P(coff), P(lens), n, P(dout), P(oo), P(ln),
                                                    P(got)) == 0
        # the GPU gather over the caller's mapped range, or the pinned staging
        assert rc.lib.enet_rc_last_host_paths(rc.ctx) & 0xF == (4 if mem == "pinned" else 1)
        assert np.array_equal(got, ln), (np.nonzero(got != ln)[0][:8], rc.last_lane_count())
        bad = []
        for i in range(n):
            src = a if which[i] == 0 else b
            want = src[0][int(src[1][i]): int(src[1][i]) + int(src[2][i])]
            if not np.array_equal(dout[int(oo[i]): int(oo[i]) + int(ln[i])], want):
                bad.append(i)
        assert not bad, bad[:8]

    buf = _pinned(total, 0xEE) if mem == "pinned" else np.full(total, 0xEE, np.uint8)
    which = np.zeros(n, np.int8)
    check(buf, fill(buf, which), which)
    which = np.ones(n, np.int8)                   # every stream rewritten by the CPU in place
    check(buf, fill(buf, which), which)
    which = (np.arange(n) % 2).astype(np.int8)    # half of them back
    check(buf, fill(buf, which), which)
    del buf                                        # a new buffer, likely on the same pages
    buf = _pinned(total, 0x11) if mem == "pinned" else np.full(total, 0x11, np.uint8)
    which = np.zeros(n, np.int8)
    check(buf, fill(buf, which), which)


@pytest.mark.parametrize("mem", ["pinned", "pageable"])
def test_back_to_back_slots_keep_bytes_past_out_len(rc, mem):
    from oracle.pyoracle import compress_batch, decompress_batch
    n, size = 4000, 1200
    d, o, l = synth.random_batch(n, size, seed=0x5A33)
    out, oo, ocap, ol = compress_batch(d, o, l, "port")
    rng = np.random.default_rng(5)
    bad = rng.choice(n, n // 8, replace=False)
    for i in bad:                                   # corrupt streams: short or failed decodes
        at = int(oo[i]) + int(rng.integers(2, max(int(ol[i]) - 1, 3)))
        out[at] ^= np.uint8(1 + rng.integers(0, 255))
    want, wo, wl = decompress_batch(out, oo, ol, l)
    assert (wl != l).sum() > 0                     # some slots are not filled
    for trial in ("corrupt", "clean"):
        if trial == "clean":
            out, oo, ocap, ol = compress_batch(d, o, l, "port")
            want, wo, wl = decompress_batch(out, oo, ol, l)
        dout = _pinned(n * size + 64, 0x3C) if mem == "pinned" else np.full(n * size + 64, 0x3C, np.uint8)
        got = np.zeros(n, np.uint32)
        l32 = l.astype(np.uint32)
        assert rc.lib.enet_rc_decompress_batch_host(rc.ctx, P(out), P(oo), P(ol), n, P(dout), P(o), P(l32),
                                                    P(got)) == 0
        assert np.array_equal(got, wl)
        paths = rc.lib.enet_rc_last_host_paths(rc.ctx) >> 4
        # one DMA of the span into a page-locked buffer only when every slot is full
        assert (paths == 2) == (trial == "clean" and mem == "pinned"), paths
        for i in range(n):
            s = int(o[i])
            assert np.array_equal(dout[s: s + int(got[i])], want[int(wo[i]): int(wo[i]) + int(wl[i])]), i
            assert (dout[s + int(got[i]): s + size] == 0x3C).all(), i


def test_slot_handoff_many_packets_per_lane(rc):
    """The record-light decoder's input hand-off on the hardware across packet
    boundaries: 4 x 65536 short random packets, so every decoding lane takes
    several packets in turn (new generations, the helper's new-packet path,
    rc_slot.h), decoded through the device entry against the oracle; the
    hand-off's check sums (rc_dec6_verify) must never disagree
    (enet_rc_debug_counter 7 counts the packets they sent to the lane kernels)."""
    import torch
    from oracle.pyoracle import compress_batch, fnv_digest
    n = 4 * 65536
    d, o, l = synth.mixed_batch(n, lo=24, hi=300, seed=0x5A34)
    want, wo, wcap, wl = compress_batch(d, o, l, "port")
    dev = lambda a, t: torch.from_numpy(np.ascontiguousarray(a)).to(t).cuda()  # noqa: E731
    din, doff, dlen = dev(d, torch.uint8), dev(o, torch.int64), dev(l, torch.int32)
    cap = (2 * dlen.to(torch.int64) + 64).to(torch.int32)
    coff = torch.zeros(n, dtype=torch.int64, device="cuda")
    coff[1:] = torch.cumsum(cap[:-1].to(torch.int64), 0)
    cout = torch.zeros(int(coff[-1] + cap[-1]), dtype=torch.uint8, device="cuda")
    clen = torch.zeros(n, dtype=torch.int32, device="cuda")
    rc.compress_batch(din, doff, dlen, cout, coff, cap, clen, max_len=int(l.max()))
    torch.cuda.synchronize()
    cl = clen.cpu().numpy().astype(np.uint32)
    assert np.array_equal(cl, wl)
    assert fnv_digest(cout.cpu().numpy(), coff.cpu().numpy().astype(np.uint64), cl) == fnv_digest(want, wo, wl)
    for _ in range(3):
        dout = torch.zeros_like(din)
        dl = torch.zeros(n, dtype=torch.int32, device="cuda")
        rc.decompress_batch(cout, coff, clen, dout, doff, dlen, dl, max_len=int(cl.max()))
        torch.cuda.synchronize()
        assert torch.equal(dl, dlen) and torch.equal(dout, din)
        assert rc.lib.enet_rc_debug_counter(rc.ctx, 7) == 0          # no hand-off sum mismatch
        assert rc.last_lane_count() == 0
