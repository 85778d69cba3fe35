"""The two-pass encoder's wide mode on the GPU (rc_enc2_wscan / rc_enc2_wcode,
rc_enc2.hip): packets with a bucket over 64 positions, whose sub-contexts
rescale (compress.c:90-112, :313-314).  Bit-exact against the oracle, through
the C ABI, on batches large enough for the lane path (small batches run on the
wave kernel).  The model the kernels follow is tests/proto/twopass.py
(scan_wide), checked on the CPU in tests/test_twopass_model.py.
"""
import os

import numpy as np
import pytest

from enet_amd import synth

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _coder(**env):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from enet_amd import RangeCoder
    env = {"ENET_RC_KERNEL": "lane3", "ENET_RC_SMALL_BATCH": "0", **env}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return RangeCoder()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _wide_packets(n, seed, max_len=1919):
    """Low-entropy packets of every shape the wide path has to get right:
    single-byte runs (one context, rescales every 127 visits), alternations,
    small alphabets, mostly-zero with random bytes, game state, lengths up to
    1919 B (the longest without a model reset) or max_len, every 11th packet
    exactly max_len long."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        k = i % 7
        ln = max_len if i % 11 == 0 else int(rng.integers(66, max_len + 1))
        if k == 0:
            p = np.full(ln, rng.integers(0, 256), np.uint8)
        elif k == 1:
            per = int(rng.integers(2, 5))
            p = np.resize(rng.integers(0, 256, per).astype(np.uint8), ln)
        elif k == 2:
            alpha = rng.integers(0, 256, int(rng.integers(2, 9))).astype(np.uint8)
            p = alpha[rng.integers(0, len(alpha), ln)]
        elif k == 3:
            p = np.where(rng.random(ln) < rng.uniform(0.5, 0.95), 0, rng.integers(0, 256, ln)).astype(np.uint8)
        elif k == 4:
            # a long run, then random bytes (dense walks, then small buckets)
            cut = int(rng.integers(1, ln))
            p = np.concatenate([np.zeros(cut, np.uint8), rng.integers(0, 256, ln - cut).astype(np.uint8)])
        elif k == 5:
            # two interleaved heavy contexts in one bucket: (0, 0) and (5, 0)
            p = np.resize(np.array([0, 0, 5, 0], np.uint8), ln)
            flip = rng.random(ln) < 0.05
            p[flip] = rng.integers(0, 256, int(flip.sum()))
        else:
            # skewed symbols inside one heavy context: many distinct values per round
            p = np.where(np.arange(ln) % 2 == 0, 0, rng.geometric(0.05, ln) % 256).astype(np.uint8)
        out.append(p.tobytes())
    return out


def _check(coder, packets, cap_fn):
    from oracle.pyoracle import compress_batch as ocompress
    d, o, l = synth.pack(packets)
    ref, roff, cap, rlen = ocompress(d, o, l, "port", cap_fn=cap_fn)
    n = len(l)
    din = torch.from_numpy(d).cuda()
    doff = torch.from_numpy(o.astype(np.int64)).cuda()
    dlen = torch.from_numpy(l.astype(np.int32)).cuda()
    coff = torch.from_numpy(roff.astype(np.int64)).cuda()
    ccap = torch.from_numpy(cap.astype(np.int32)).cuda()
    cout = torch.zeros(int(cap.sum()) + 1, dtype=torch.uint8, device="cuda")
    clen = torch.zeros(n, dtype=torch.int32, device="cuda")
    coder.compress_batch(din, doff, dlen, cout, coff, ccap, clen, max_len=int(l.max()))
    torch.cuda.synchronize()
    gl = clen.cpu().numpy().astype(np.uint32)
    bad = np.nonzero(gl != rlen)[0]
    assert bad.size == 0, [(int(i), int(l[i]), int(gl[i]), int(rlen[i])) for i in bad[:8]]
    go = cout.cpu().numpy()
    for i in range(n):
        a, b = int(roff[i]), int(roff[i]) + int(rlen[i])
        assert np.array_equal(go[a:b], ref[a:b]), (i, int(l[i]))


def test_wide_packets_vs_oracle():
    c = _coder()
    pk = _wide_packets(3000, 11)
    _check(c, pk, lambda n: 2 * n + 64)
    assert c.last_lane_count() == 0                   # every packet on the wide path
    _check(c, pk, lambda n: n)                        # protocol mode: outLimit = N (overflows included)
    c.close()


@pytest.mark.parametrize("slow", ["0", "1"])
def test_wide_small_layout_vs_oracle(slow):
    """Launches whose packets are at most 1216 B take rc_enc2_wscan_s, whose
    LDS layout is sized for them (WScanLdsT<1216>: u16 position lists, the
    window's bytes exactly as long as such a packet at any alignment needs):
    the adversarial shapes at every length up to 1216 and back-to-back
    offsets (all 16 alignments), with and without the lane-order shortcut."""
    c = _coder(ENET_RC_ENC2_SLOW=slow)
    pk = _wide_packets(3000, 21, max_len=1216)
    assert max(len(p) for p in pk) == 1216
    _check(c, pk, lambda n: 2 * n + 64)
    assert c.last_lane_count() == 0
    _check(c, pk, lambda n: n)
    c.close()


def test_wide_gamestate_and_random_mixed():
    c = _coder()
    d, o, l = synth.gamestate_batch(2048, 1200)
    pk = [d[int(o[i]): int(o[i]) + 1200].tobytes() for i in range(2048)]
    rng = np.random.default_rng(3)
    pk += [rng.integers(0, 256, int(rng.integers(1, 1920)), dtype=np.uint8).tobytes() for _ in range(1024)]
    rng.shuffle(pk)
    _check(c, pk, lambda n: 2 * n + 64)
    assert c.last_lane_count() == 0
    c.close()


def test_wide_slow_path_full_peeling():
    """ENET_RC_ENC2_SLOW=1: no reliance on lane-ordered LDS atomics (every
    key peeled with ballots)."""
    c = _coder(ENET_RC_ENC2_SLOW="1")
    _check(c, _wide_packets(1500, 12), lambda n: 2 * n + 64)
    c.close()


def test_wide_stream_overflow_goes_to_lanes():
    """A wide stream for only a few packets (ENET_RC_ENC2_WIDE_MB=1): the rest
    of the listed packets take the lane kernels, still bit-exact."""
    c = _coder(ENET_RC_ENC2_WIDE_MB="1")
    d, o, l = synth.gamestate_batch(3000, 1200)
    pk = [d[int(o[i]): int(o[i]) + 1200].tobytes() for i in range(3000)]
    _check(c, pk, lambda n: 2 * n + 64)
    assert 0 < c.last_lane_count() < 3000
    c.close()


def test_wide_across_stream_chunks():
    """Record-stream chunks (ENET_RC_ENC2_STREAM_MB=8): the wide list is per
    chunk."""
    c = _coder(ENET_RC_ENC2_STREAM_MB="8")
    pk = _wide_packets(2500, 13)
    _check(c, pk, lambda n: 2 * n + 64)
    assert c.last_lane_count() == 0
    c.close()


def test_wide_off_takes_lanes():
    c = _coder(ENET_RC_ENC2_WIDE="0")
    d, o, l = synth.gamestate_batch(2048, 1200)
    pk = [d[int(o[i]): int(o[i]) + 1200].tobytes() for i in range(2048)]
    _check(c, pk, lambda n: 2 * n + 64)
    assert c.last_lane_count() == 2048
    c.close()


def _long_wide_packets(n, seed):
    """Wide packets of 1920-4096 bytes (a bucket over 64 positions): low-entropy
    ones that never reach compress.c's model reset within 4096 bytes (game
    state, mostly-zero), and skewed random ones that reset once or twice
    (compress.c:148-157 at 4094 nodes: zeros with random bytes between them
    make ~2 nodes per random byte)."""
    rng = np.random.default_rng(seed)
    d, o, l = synth.gamestate_batch(max(1, n // 4), 4096)
    out = [d[int(o[i]): int(o[i]) + int(l[i])].tobytes()[: int(rng.integers(1920, 4097))] for i in range(len(l))]
    while len(out) < n:
        ln = int(rng.integers(1920, 4097))
        z = rng.uniform(0.25, 0.6) if len(out) % 2 else rng.uniform(0.6, 0.95)
        out.append(np.where(rng.random(ln) < z, 0, rng.integers(0, 256, ln)).astype(np.uint8).tobytes())
    return out


def test_wide_model_reset_vs_oracle():
    """The wide mode through the model reset (compress.c:148-157): windows at
    the reset byte, the code pass clearing its root there; every packet stays
    on the wide path, bit-exact, both outLimit modes."""
    from tests.proto.twopass import scan_wide
    c = _coder()
    pk = _long_wide_packets(1200, 21)
    # (the generator does reach the reset: the model restated in tests/proto/twopass.py)
    assert sum(1 for p in pk[301:341] for rec in scan_wide(p, max_len=4096) if rec[3]) > 0
    _check(c, pk, lambda n: 2 * n + 64)
    assert c.last_lane_count() == 0
    _check(c, pk, lambda n: n)
    c.close()


def test_wide_4096_gamestate_full_batch():
    """65536 game-state packets of 4096 bytes: every packet on the wide path
    (last_lane_count 0), bit-exact against the oracle on a sample and the round
    trip on all."""
    from oracle.pyoracle import compress_batch as ocompress
    c = _coder()
    d, o, l = synth.gamestate_batch(65536, 4096)
    n = len(l)
    din = torch.from_numpy(d).cuda()
    doff = torch.from_numpy(o.astype(np.int64)).cuda()
    dlen = torch.from_numpy(l.astype(np.int32)).cuda()
    cap = (2 * dlen.to(torch.int64) + 64).to(torch.int32)
    coff = torch.zeros(n, dtype=torch.int64, device="cuda")
    coff[1:] = torch.cumsum(cap[:-1].to(torch.int64), 0)
    cout = torch.zeros(int(coff[-1] + cap[-1]), dtype=torch.uint8, device="cuda")
    clen = torch.zeros(n, dtype=torch.int32, device="cuda")
    c.compress_batch(din, doff, dlen, cout, coff, cap, clen, max_len=4096)
    torch.cuda.synchronize()
    assert c.last_lane_count() == 0 and c.last_exact_count() == 0
    cl = clen.cpu().numpy().astype(np.uint32)
    co = coff.cpu().numpy()
    cb = cout.cpu().numpy()
    sel = np.arange(0, n, 97)
    ref, roff, rcap, rlen = ocompress(np.concatenate([d[int(o[i]): int(o[i]) + 4096] for i in sel]),
                                      (np.arange(len(sel)) * 4096).astype(np.uint64),
                                      np.full(len(sel), 4096, np.uint32), "port")
    for k, i in enumerate(sel):
        assert int(cl[i]) == int(rlen[k]), i
        assert np.array_equal(cb[int(co[i]): int(co[i]) + int(cl[i])], ref[int(roff[k]): int(roff[k]) + int(rlen[k])]), i
    back = torch.zeros_like(din)
    bl = torch.zeros(n, dtype=torch.int32, device="cuda")
    c.decompress_batch(cout, coff, clen, back, doff, dlen, bl, max_len=int(cl.max()))
    torch.cuda.synchronize()
    assert torch.equal(bl, dlen) and torch.equal(back, din)
    c.close()
