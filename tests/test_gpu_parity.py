"""Parity of the HIP path (through the C ABI) with the reference.

Small cases: against the committed golden fixtures produced by the real
compress.c.  Full BASELINE sizes: against the reference digests committed in
tests/golden/digests.json plus round-trip identity.
Bit-exact throughout: return value and the returned bytes.  (On a 0 return
the reference leaves unspecified partial bytes in outData; only the return
value is compared there, as the protocol discards the buffer, protocol.c:1067.)
"""
import numpy as np
import pytest

from enet_amd import synth
from tests import golden_io

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


VARIANTS = {
    # default: two-pass encoder (rc_enc2.hip) and record-light decoder with its
    # check, its input through LDS slots (rc_dec6.hip rc_decompress_dec6s, rc_slot.h),
    # in front of the v3 lane kernels (rc_lane3.hip)
    "lane3": {"ENET_RC_KERNEL": "lane3"},
    # the two-pass encoder's slow paths forced (every position exceptional,
    # every bucket sorted and re-walked: what a device without lane-ordered
    # LDS atomics would take)
    "enc2-slow": {"ENET_RC_KERNEL": "lane3", "ENET_RC_ENC2_SLOW": "1"},
    # the v3 lane kernels alone, both directions
    "lane3-only": {"ENET_RC_KERNEL": "lane3", "ENET_RC_ENC2": "0", "ENET_RC_DEC4": "0"},
}


@pytest.fixture(scope="module", params=list(VARIANTS))
def coder(request):
    """Every test runs on each kernel configuration, selected by environment
    when the coder context is created."""
    import os
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from enet_amd import RangeCoder
    env = VARIANTS[request.param]
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        c = RangeCoder()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    c.variant = request.param
    yield c
    c.close()


def _dev(a, dtype):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dtype).cuda()


def _pack(packets):
    d, o, l = synth.pack(packets)
    if d.size == 0:
        d = np.zeros(1, np.uint8)
    return d, o, l


def _run(coder, decompress, packets, caps, max_len=None, max_out=0):
    d, o, l = _pack(packets)
    caps = np.asarray(caps, dtype=np.int64)
    out_off = np.zeros(len(caps), np.int64)
    out_off[1:] = np.cumsum(caps[:-1])
    out = torch.zeros(int(caps.sum()) + 1, dtype=torch.uint8, device="cuda")
    out_len = torch.zeros(len(caps), dtype=torch.int32, device="cuda")
    args = (_dev(d, torch.uint8), _dev(o, torch.int64), _dev(l, torch.int32), out,
            _dev(out_off, torch.int64), _dev(caps, torch.int32), out_len)
    ml = int(l.max()) if max_len is None and len(l) else (max_len or 0)
    if decompress:
        coder.decompress_batch(*args, max_len=ml, max_out=max_out)
    else:
        coder.compress_batch(*args, max_len=ml)
    torch.cuda.synchronize()
    ol = out_len.cpu().numpy().astype(np.int64)
    ob = out.cpu().numpy()
    return [(int(ol[i]), ob[out_off[i]: out_off[i] + ol[i]].tobytes()) for i in range(len(caps))]


def test_compress_fixtures(coder):
    cases = [c for c in golden_io.compress_cases() if c["in_limit"] == len(c["input"])]
    res = _run(coder, False, [c["input"] for c in cases], [c["out_limit"] for c in cases])
    bad = [(len(c["input"]), c["out_limit"], r[0], c["ret"]) for c, r in zip(cases, res)
           if r[0] != c["ret"] or (c["ret"] and r[1] != c["expect"])]
    assert not bad, bad[:10]


def test_decompress_fixtures_incl_garbage(coder):
    cases = golden_io.decompress_cases()
    res = _run(coder, True, [c["input"] for c in cases], [c["out_limit"] for c in cases])
    bad = [(i, len(c["input"]), r[0], c["ret"]) for i, (c, r) in enumerate(zip(cases, res))
           if r[0] != c["ret"] or (c["ret"] and r[1] != c["expect"])]
    assert not bad, bad[:10]
    # the corrupt streams exercise the exact (binary-tree) path
    assert coder.last_exact_count() > 0


def test_gather_fixtures_per_call(coder):
    for c in golden_io.gather_cases():
        r = coder.compress_gather(c["backing"], c["spans"], c["in_limit"], c["out_limit"])
        assert r[0] == c["ret"], c["spans"][:4]
        if c["ret"]:
            assert r[1] == c["expect"]


def test_per_call_reference_surface(coder):
    cases = golden_io.compress_cases()[:60]
    for c in cases:
        r = coder.compress(c["input"], out_limit=c["out_limit"], in_limit=c["in_limit"])
        assert r[0] == c["ret"]
        if c["ret"]:
            assert r[1] == c["expect"]
    for c in golden_io.decompress_cases()[::97]:
        r = coder.decompress(c["input"], c["out_limit"])
        assert r[0] == c["ret"]
        if c["ret"]:
            assert r[1] == c["expect"]
    assert coder.compress(b"", in_limit=0) == (0, b"")
    assert coder.decompress(b"", 100) == (0, b"")


def _digest_roundtrip(coder, name, batch, lanes=None):
    """Digest + round trip at full size.  lanes = (compress, decompress): the
    packets the fast kernels (rc_enc2.hip, rc_dec4.hip) must hand to the lane
    kernels on the default configuration; a fast path that starts bailing
    silently would pass every parity check and only lose speed."""
    from oracle.pyoracle import fnv_digest
    d, o, l = batch
    g = golden_io.digests()[name]
    n = len(l)
    din, doff, dlen = _dev(d, torch.uint8), _dev(o, torch.int64), _dev(l, torch.int32)
    cap = (2 * dlen.to(torch.int64) + 64).to(torch.int32)
    coff = torch.zeros(n, dtype=torch.int64, device="cuda")
    coff[1:] = torch.cumsum(cap[:-1].to(torch.int64), 0)
    cout = torch.empty(int(coff[-1] + cap[-1]), dtype=torch.uint8, device="cuda")
    clen = torch.zeros(n, dtype=torch.int32, device="cuda")
    coder.compress_batch(din, doff, dlen, cout, coff, cap, clen, max_len=int(l.max()))
    torch.cuda.synchronize()
    routed = getattr(coder, "variant", "") == "lane3" and lanes is not None
    if routed and lanes[0] is not None:
        assert coder.last_lane_count() == lanes[0], "encoder fast path hand-off"
        assert coder.last_exact_count() == 0
    cl = clen.cpu().numpy().astype(np.uint32)
    assert int(cl.sum()) == g["out_bytes"]
    assert fnv_digest(cout.cpu().numpy(), coff.cpu().numpy().astype(np.uint64), cl) == g["digest"]
    # decompress back
    dout = torch.empty_like(din)
    dl = torch.zeros(n, dtype=torch.int32, device="cuda")
    coder.decompress_batch(cout, coff, clen, dout, doff, dlen, dl, max_len=int(cl.max()))
    torch.cuda.synchronize()
    if routed and lanes[1] is not None:
        assert coder.last_lane_count() == lanes[1], "decoder fast path hand-off"
        assert coder.last_exact_count() == 0
    assert torch.equal(dl, dlen)
    assert torch.equal(dout, din)


def test_c1_digest(coder):
    _digest_roundtrip(coder, "C1_random_4096x256", synth.random_batch(4096, 256))


def test_c2_digest_full_size(coder):
    # every C2 packet stays on the fast kernels, both directions
    _digest_roundtrip(coder, "C2_random_65536x1200", synth.random_batch(65536, 1200), lanes=(0, 0))


def test_c3_digest_full_size(coder):
    # game state: every packet on the encoder's wide mode; the decoder hands
    # them all to the lane kernels (buckets over its capacity)
    _digest_roundtrip(coder, "C3_gamestate_65536x1200", synth.gamestate_batch(65536, 1200), lanes=(0, 65536))


def test_c4_mixed_sizes_vs_oracle(coder):
    from oracle.pyoracle import compress_batch as ocompress, fnv_digest
    d, o, l = synth.mixed_batch(1 << 15)
    out, oo, cap, ol = ocompress(d, o, l, "port")
    packets = [d[int(o[i]): int(o[i]) + int(l[i])].tobytes() for i in range(len(l))]
    res = _run(coder, False, packets, [int(c) for c in cap])
    if getattr(coder, "variant", "") == "lane3":                 # random C4 packets: all on the fast encoder
        assert coder.last_lane_count() == 0 and coder.last_exact_count() == 0
    gl = np.array([r[0] for r in res], np.uint32)
    assert np.array_equal(gl, ol)
    blob = np.frombuffer(b"".join(r[1] for r in res), np.uint8)
    goff = np.concatenate([[0], np.cumsum(gl[:-1].astype(np.uint64))]).astype(np.uint64)
    assert fnv_digest(blob, goff, gl) == fnv_digest(out, oo, ol)
    back = _run(coder, True, [r[1] for r in res], [len(p) for p in packets])
    if getattr(coder, "variant", "") == "lane3":                 # ... and on the fast decoder
        assert coder.last_lane_count() == 0 and coder.last_exact_count() == 0
    assert all(b == (len(p), p) for b, p in zip(back, packets))


def test_max_len_below_packet_lengths(coder):
    """A batch's max_len hint below some of its packets' lengths: the
    encoder's record slots are sized by max_len, so the longer packets must
    go to the lane kernels (whose arena, also sized by max_len, sends what
    outgrows it to the exact path) -- never past their slot.  Bit-exact
    against the oracle, then back with the same kind of hint."""
    from oracle.pyoracle import Coder
    port = Coder("port")
    rng = np.random.default_rng(404)
    pk = []
    for i in range(8192):
        n = int(rng.integers(1, 1900)) if i % 3 else int(rng.integers(1, 300))
        alpha = int(rng.choice([3, 40, 256]))
        pk.append(rng.integers(0, alpha, size=n).astype(np.uint8).tobytes())
    caps = [2 * len(p) + 64 for p in pk]
    res = _run(coder, False, pk, caps, max_len=300)
    want = [port.compress(p, out_limit=c) for p, c in zip(pk, caps)]
    bad = [i for i, (r, w) in enumerate(zip(res, want)) if r != w]
    assert not bad, bad[:10]
    back = _run(coder, True, [r[1] for r in res], [len(p) for p in pk], max_len=200)
    bad = [i for i, (b, p) in enumerate(zip(back, pk)) if b != (len(p), p)]
    assert not bad, bad[:10]


def test_protocol_out_limit_mode(coder):
    # ENet calls compress with outLimit = inLimit (protocol.c:1690-1695)
    from oracle.pyoracle import Coder
    port = Coder("port")
    pk = [synth.random_bytes(1200, s).tobytes() for s in range(64)]
    gd, go, gl = synth.gamestate_batch(64, 1200)
    pk += [gd[int(go[i]): int(go[i]) + 1200].tobytes() for i in range(64)]
    res = _run(coder, False, pk, [len(p) for p in pk])
    for p, r in zip(pk, res):
        assert r == port.compress(p, out_limit=len(p))


def test_no_write_past_out_cap(coder):
    """A packet whose output does not fit returns 0 (compress.c:116-117) and
    writes nothing past its capacity: every output slot is followed by a
    64-B canary that must survive.  Caps below, at and just above what each
    packet needs, misaligned slot starts."""
    from oracle.pyoracle import Coder
    port = Coder("port")
    rng = np.random.default_rng(23)
    pk = [synth.random_bytes(int(n), 40 + i).tobytes() for i, n in enumerate(rng.integers(1, 1500, 768))]
    pk += [rng.integers(0, 7, size=int(n)).astype(np.uint8).tobytes() for n in rng.integers(1, 1500, 256)]
    need = [port.compress(p, out_limit=2 * len(p) + 64)[0] for p in pk]
    caps = [max(1, int(c + rng.integers(-20, 3))) for c in need]
    d, o, l = _pack(pk)
    caps = np.asarray(caps, np.int64)
    gap = 64 + 3
    out_off = np.zeros(len(caps), np.int64)
    out_off[1:] = np.cumsum(caps[:-1] + gap)
    total = int(out_off[-1] + caps[-1] + gap)
    out = torch.full((total,), 0xA5, dtype=torch.uint8, device="cuda")
    out_len = torch.zeros(len(caps), dtype=torch.int32, device="cuda")
    coder.compress_batch(_dev(d, torch.uint8), _dev(o, torch.int64), _dev(l, torch.int32), out,
                         _dev(out_off, torch.int64), _dev(caps, torch.int32), out_len, max_len=int(l.max()))
    torch.cuda.synchronize()
    ob, ol = out.cpu().numpy(), out_len.cpu().numpy()
    for i, p in enumerate(pk):
        e = port.compress(p, out_limit=int(caps[i]))
        assert int(ol[i]) == e[0], i
        if e[0]:
            assert ob[out_off[i]: out_off[i] + e[0]].tobytes() == e[1], i
        canary = ob[out_off[i] + caps[i]: out_off[i] + caps[i] + gap]
        assert (canary == 0xA5).all(), (i, int(caps[i]), need[i])


def test_long_packets_and_model_reset(coder):
    from oracle.pyoracle import Coder
    port = Coder("port")
    pk = [synth.de_bruijn_bytes(n) for n in (1919, 1920, 2600, 4096)]
    pk += [synth.random_bytes(n, 5 + n).tobytes() for n in (2000, 3000, 4096)]
    pk += [b"\0" * 4096, (synth.random_bytes(4096, 9) % 3).astype(np.uint8).tobytes()]
    caps = [2 * len(p) + 64 for p in pk]
    res = _run(coder, False, pk, caps)
    for p, c, r in zip(pk, caps, res):
        assert r == port.compress(p, out_limit=c)
    back = _run(coder, True, [r[1] for r in res], [4096] * len(res))
    for p, r in zip(pk, back):
        assert r == (len(p), p)


def test_mtu_packets_model_reset_on_fast_decoder(coder):
    """Random packets of 1920-4096 bytes go through compress.c's model reset
    (4094 nodes, compress.c:148-157) once or twice: the record-light decoder
    resets its model itself (rc_dec6.hip reset6) and its check counts bigrams
    per model segment, so on the default variants none is left to the lane
    kernels.  Bit-exact against the oracle."""
    from oracle.pyoracle import Coder
    port = Coder("port")
    rng = np.random.default_rng(0x4D54)
    sizes = [4096] * 64 + [int(x) for x in rng.integers(1920, 4097, size=448)]
    pk = [rng.integers(0, 256, size=n, dtype=np.uint8).tobytes() for n in sizes]
    comp = [port.compress(p, 2 * len(p) + 64)[1] for p in pk]
    back = _run(coder, True, comp, [4096] * len(comp), max_len=max(len(c) for c in comp))
    if getattr(coder, "variant", "") == "lane3":
        assert coder.last_lane_count() == 0 and coder.last_exact_count() == 0
    assert all(b == (len(p), p) for b, p in zip(back, pk))
    # output limits inside the second segment
    back = _run(coder, True, comp[:64], [3000] * 64, max_len=max(len(c) for c in comp))
    assert all(b == port.decompress(c, 3000) for b, c in zip(back, comp[:64]))


def test_mtu_packets_model_reset_on_fast_encoder(coder):
    """Packets of 1920-4096 bytes reach compress.c's model reset (4094 nodes,
    compress.c:148-157): the two-pass encoder scans them in windows, one per
    model segment (rc_enc2.hip reset_after), and its code pass resets the
    root where a record carries kRst; on the default variants none is left
    to the lane kernels.  Random, de Bruijn and small-alphabet packets
    (several resets, resets late in a window), bit-exact against the oracle,
    and back."""
    from oracle.pyoracle import Coder
    port = Coder("port")
    rng = np.random.default_rng(0x454E)
    sizes = [4096] * 96 + [1920, 1921, 2047, 2048, 2049, 3071, 4095] + [int(x) for x in rng.integers(1920, 4097, size=320)]
    pk = [rng.integers(0, 256, size=n, dtype=np.uint8).tobytes() for n in sizes]
    narrow = len(pk)
    pk += [synth.de_bruijn_bytes(n) for n in (1920, 2600, 4096)]
    pk += [rng.integers(0, 40, size=4096, dtype=np.uint8).tobytes() for _ in range(8)]
    caps = [2 * len(p) + 64 for p in pk]
    res = _run(coder, False, pk[:narrow], caps[:narrow])
    if getattr(coder, "variant", "") == "lane3":
        assert coder.last_lane_count() == 0 and coder.last_exact_count() == 0
    res += _run(coder, False, pk[narrow:], caps[narrow:])
    for p, c, r in zip(pk, caps, res):
        assert r == port.compress(p, out_limit=c), len(p)
    # output limits that cut a packet inside its second model segment
    cut = _run(coder, False, pk[:32], [2100] * 32)
    for p, r in zip(pk[:32], cut):
        assert r == port.compress(p, out_limit=2100)
    back = _run(coder, True, [r[1] for r in res], [4096] * len(res), max_len=max(len(r[1]) for r in res))
    assert all(b == (len(p), p) for b, p in zip(back, pk))


def test_random_fuzz_vs_oracle(coder):
    from oracle.pyoracle import Coder
    port = Coder("port")
    rng = np.random.default_rng(11)
    pk = []
    for _ in range(2000):
        n = int(rng.integers(1, 1500))
        alpha = int(rng.choice([1, 2, 3, 7, 40, 256]))
        pk.append(rng.integers(0, alpha, size=n).astype(np.uint8).tobytes())
    caps = [int(rng.choice([len(p), 2 * len(p) + 64, len(p) // 3 + 1])) for p in pk]
    res = _run(coder, False, pk, caps)
    for p, c, r in zip(pk, caps, res):
        e = port.compress(p, out_limit=c)
        assert r[0] == e[0] and (e[0] == 0 or r[1] == e[1])
    garbage = [rng.integers(0, 256, size=int(rng.integers(1, 400)), dtype=np.uint8).tobytes() for _ in range(2000)]
    res = _run(coder, True, garbage, [2048] * len(garbage))
    for g, r in zip(garbage, res):
        e = port.decompress(g, 2048)
        assert r[0] == e[0] and (e[0] == 0 or r[1] == e[1])


def test_corrupted_streams_vs_oracle(coder):
    """Valid streams of random packets with a few bytes flipped: the decode
    stays on the record-light decoder's common steps for a while, then
    escapes past symbols its contexts hold (compress.c:606-610), which only
    its bigram-count check (rc_dec6_verify) can tell.  Every result, the
    packets the check sent to the lane kernels included, matches the oracle."""
    from oracle.pyoracle import Coder
    port = Coder("port")
    rng = np.random.default_rng(29)
    streams = []
    for _ in range(3000):
        n = int(rng.integers(200, 1300))
        p = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        r, c = port.compress(p, 2 * n + 64)
        b = bytearray(c)
        for _ in range(int(rng.integers(1, 4))):
            j = int(rng.integers(len(b) // 4, len(b)))
            b[j] ^= 1 << int(rng.integers(0, 8))
        streams.append(bytes(b))
    caps = [int(rng.choice([1400, 4096])) for _ in streams]
    res = _run(coder, True, streams, caps)
    bad = [i for i, (g, c, r) in enumerate(zip(streams, caps, res))
           if (lambda e: r[0] != e[0] or (e[0] and r[1] != e[1]))(port.decompress(g, c))]
    assert not bad, bad[:10]


def test_check_on_unaligned_outputs_vs_oracle(coder):
    """The decoder's check (rc_dec6_verify) reads each output as aligned dwords
    from the one holding its first byte: outputs at every offset mod 4 (caps
    n + 0..3, 5, 7), packets of 1 to 1500 bytes, valid streams (none left to
    the lane kernels on the default variants) and bit-flipped ones, against
    the oracle."""
    from oracle.pyoracle import Coder
    port = Coder("port")
    rng = np.random.default_rng(0x5646)
    pk = [rng.integers(0, 256, size=int(rng.integers(1, 1501)), dtype=np.uint8).tobytes() for _ in range(600)]
    comp = [port.compress(p, 2 * len(p) + 64)[1] for p in pk]
    caps = [len(p) + int(rng.choice([0, 1, 2, 3, 5, 7])) for p in pk]
    back = _run(coder, True, comp, caps)
    if getattr(coder, "variant", "") == "lane3":
        assert coder.last_lane_count() == 0 and coder.last_exact_count() == 0
    assert all(b == (len(p), p) for b, p in zip(back, pk))
    flipped = []
    for c in comp[:300]:
        b = bytearray(c)
        j = int(rng.integers(len(b) // 4, len(b))) if len(b) > 4 else len(b) - 1
        b[j] ^= 1 << int(rng.integers(0, 8))
        flipped.append(bytes(b))
    res = _run(coder, True, flipped, caps[:300])
    bad = [i for i, (g, c, r) in enumerate(zip(flipped, caps, res))
           if (lambda e: r[0] != e[0] or (e[0] and r[1] != e[1]))(port.decompress(g, c))]
    assert not bad, bad[:10]


@pytest.fixture(scope="module")
def wave_coder():
    """The one-packet-per-wavefront kernels (ENET_RC_KERNEL=wave), kept as an
    alternative path; the default is one packet per lane."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import os
    from enet_amd import RangeCoder
    os.environ["ENET_RC_KERNEL"] = "wave"
    try:
        c = RangeCoder()
    finally:
        del os.environ["ENET_RC_KERNEL"]
    yield c
    c.close()


def test_wave_kernel_fixtures(wave_coder):
    test_compress_fixtures(wave_coder)
    test_decompress_fixtures_incl_garbage(wave_coder)
    test_c1_digest(wave_coder)
    test_long_packets_and_model_reset(wave_coder)
    test_random_fuzz_vs_oracle(wave_coder)


def test_small_batches_vs_oracle(coder):
    """Batches that fit on the chip at one wavefront per packet (the
    per-datagram calls among them) run on the wavefront-per-packet kernel
    (rc_kernels.hip launch): bit-exact, all sizes, several wavefronts per CU
    (n > 256 CUs), and both sides of the decoder's 512-packet limit."""
    from oracle.pyoracle import Coder
    port = Coder("port")
    rng = np.random.default_rng(31)
    for n, top in ((1, 4097), (7, 4097), (64, 4097), (300, 1401), (512, 1401), (513, 1401)):
        pk = [rng.integers(0, int(rng.choice([2, 17, 256])), size=int(rng.integers(1, top)),
                           dtype=np.uint8).tobytes() for _ in range(n)]
        caps = [2 * len(p) + 64 for p in pk]
        res = _run(coder, False, pk, caps)
        assert res == [port.compress(p, out_limit=c) for p, c in zip(pk, caps)]
        back = _run(coder, True, [r[1] for r in res], [len(p) for p in pk])
        assert back == [(len(p), p) for p in pk]


def test_host_pointer_batches_large(coder):
    """enet_rc_{compress,decompress}_batch_host on a batch large enough for the
    chunked staging copies, device-side packing and chunked D2H (rc_host.c
    run_host, rc_pack.hip): bit-exact against the oracle, ragged offsets."""
    import ctypes as C
    from oracle.pyoracle import compress_batch as ocompress, fnv_digest
    d, o, l = synth.mixed_batch(30000)          # > 16 MB each way: the chunked copies
    lib = coder.lib
    n = len(l)
    ln = l.astype(np.uint32)
    cap = (2 * ln.astype(np.int64) + 64).astype(np.uint32)
    coff = np.zeros(n, np.uint64)
    coff[1:] = np.cumsum(cap[:-1].astype(np.uint64) + 3)          # gaps: slots not back to back
    cout = np.zeros(int(coff[-1] + cap[-1]) + 16, np.uint8)
    clen = np.zeros(n, np.uint32)
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    assert lib.enet_rc_compress_batch_host(coder.ctx, p(d), p(o), p(ln), n, p(cout), p(coff), p(cap), p(clen)) == 0
    want, wo, wcap, wl = ocompress(d, o, l, "port")
    assert np.array_equal(clen, wl)
    assert fnv_digest(cout, coff, clen) == fnv_digest(want, wo, wl)
    dout = np.zeros(int(o[-1]) + int(l[-1]) + 16, np.uint8)
    dlen = np.zeros(n, np.uint32)
    assert lib.enet_rc_decompress_batch_host(coder.ctx, p(cout), p(coff), p(clen), n, p(dout), p(o), p(ln),
                                             p(dlen)) == 0
    bad = [(i, int(ln[i]), int(dlen[i]), int(clen[i])) for i in np.nonzero(dlen != ln)[0][:8]]
    assert not bad, (coder.last_lane_count(), coder.last_exact_count(), bad)
    wrong = [i for i in range(n) if not np.array_equal(dout[int(o[i]): int(o[i]) + int(ln[i])],
                                                       d[int(o[i]): int(o[i]) + int(ln[i])])]
    assert not wrong, (coder.last_lane_count(), wrong[:8])


@pytest.mark.parametrize("pieces", [3, 4])
def test_host_pointer_batches_pieces(pieces):
    """ENET_RC_HOST_SPLIT=k: a large host batch in k pieces on k contexts of
    the device (rc_host.c run_host_split: each piece's input DMA after the
    previous piece's), at equal shares of the input bytes; ragged packets,
    bit-exact against the oracle both ways."""
    import os
    import ctypes as C
    from enet_amd import RangeCoder
    from oracle.pyoracle import compress_batch as ocompress, fnv_digest
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    old = os.environ.get("ENET_RC_HOST_SPLIT")
    os.environ["ENET_RC_HOST_SPLIT"] = str(pieces)
    try:
        c = RangeCoder()
    finally:
        if old is None:
            os.environ.pop("ENET_RC_HOST_SPLIT", None)
        else:
            os.environ["ENET_RC_HOST_SPLIT"] = old
    try:
        d, o, l = synth.mixed_batch(50000, seed=29)
        lib = c.lib
        n = len(l)
        ln = l.astype(np.uint32)
        cap = (2 * ln.astype(np.int64) + 64).astype(np.uint32)
        coff = np.zeros(n, np.uint64)
        coff[1:] = np.cumsum(cap[:-1].astype(np.uint64) + 3)
        cout = np.zeros(int(coff[-1] + cap[-1]) + 16, np.uint8)
        clen = np.zeros(n, np.uint32)
        p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
        assert lib.enet_rc_compress_batch_host(c.ctx, p(d), p(o), p(ln), n, p(cout), p(coff), p(cap), p(clen)) == 0
        # (at most one piece per hardware queue but the default stream's)
        queues = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
        pieces = min(pieces, max(queues - 1, 1))
        assert lib.enet_rc_last_split(c.ctx) == pieces
        assert lib.enet_rc_config_flags(c.ctx) & 0x80000000 == 0
        want, wo, wcap, wl = ocompress(d, o, l, "port")
        assert np.array_equal(clen, wl)
        assert fnv_digest(cout, coff, clen) == fnv_digest(want, wo, wl)
        dout = np.zeros(int(o[-1]) + int(l[-1]) + 16, np.uint8)
        dlen = np.zeros(n, np.uint32)
        assert lib.enet_rc_decompress_batch_host(c.ctx, p(cout), p(coff), p(clen), n, p(dout), p(o), p(ln),
                                                 p(dlen)) == 0
        assert lib.enet_rc_last_split(c.ctx) == pieces
        assert np.array_equal(dlen, ln)
        assert np.array_equal(dout[: d.size], d)
    finally:
        c.close()


def test_host_pointer_batches_pieces_ragged():
    """Split host batches (three pieces, rc_host.c run_host_split) on a ragged
    batch: 52100 packets of 0-2000 B (every 50th empty, a packet count that
    is no multiple of the 2048-packet piece groups), inputs in gapped slots
    both ways and decompress outputs in gapped slots too (the slot-copy
    result path instead of the one-DMA one); bit-exact against the oracle."""
    import os
    import ctypes as C
    from enet_amd import RangeCoder
    from oracle.pyoracle import compress_batch as ocompress, fnv_digest
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    old = os.environ.get("ENET_RC_HOST_SPLIT")
    os.environ["ENET_RC_HOST_SPLIT"] = "3"
    try:
        c = RangeCoder()
    finally:
        if old is None:
            os.environ.pop("ENET_RC_HOST_SPLIT", None)
        else:
            os.environ["ENET_RC_HOST_SPLIT"] = old
    try:
        n = 52100
        rng = np.random.default_rng(31)
        l = rng.integers(0, 2001, n).astype(np.uint32)
        l[::50] = 0
        gap = rng.integers(0, 40, n).astype(np.uint64)
        o = np.zeros(n, np.uint64)
        o[1:] = np.cumsum(l[:-1].astype(np.uint64) + gap[:-1])
        d = rng.integers(0, 256, int(o[-1] + l[-1]) + 16, dtype=np.uint8)
        d[: d.size // 8] //= 16                      # (a low-entropy part: wide and lane paths too)
        lib = c.lib
        cap = (2 * l.astype(np.int64) + 64).astype(np.uint32)
        coff = np.zeros(n, np.uint64)
        coff[1:] = np.cumsum(cap[:-1].astype(np.uint64) + 7)
        cout = np.zeros(int(coff[-1] + cap[-1]) + 16, np.uint8)
        clen = np.zeros(n, np.uint32)
        p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
        assert lib.enet_rc_compress_batch_host(c.ctx, p(d), p(o), p(l), n, p(cout), p(coff), p(cap), p(clen)) == 0
        queues = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
        assert lib.enet_rc_last_split(c.ctx) == min(3, max(queues - 1, 1))
        want, wo, wcap, wl = ocompress(d, o, l, "port")
        assert np.array_equal(clen, wl)
        assert fnv_digest(cout, coff, clen) == fnv_digest(want, wo, wl)
        # decompress into gapped slots (a slot a packet fills exactly, 5 spare bytes between)
        doff = np.zeros(n, np.uint64)
        doff[1:] = np.cumsum(l[:-1].astype(np.uint64) + 5)
        dout = np.full(int(doff[-1] + l[-1]) + 16, 0xAB, np.uint8)
        dlen = np.zeros(n, np.uint32)
        assert lib.enet_rc_decompress_batch_host(c.ctx, p(cout), p(coff), p(clen), n, p(dout), p(doff), p(l),
                                                 p(dlen)) == 0
        assert lib.enet_rc_last_split(c.ctx) == min(3, max(queues - 1, 1))
        assert np.array_equal(dlen, l)
        bad = [i for i in range(n) if not np.array_equal(dout[int(doff[i]): int(doff[i]) + int(l[i])],
                                                         d[int(o[i]): int(o[i]) + int(l[i])])]
        assert not bad, bad[:8]
        # the gaps between slots are untouched (results go exactly to out_len bytes of each slot)
        mask = np.ones(dout.size, bool)
        for i in range(n):
            mask[int(doff[i]): int(doff[i]) + int(l[i])] = False
        assert np.all(dout[mask] == 0xAB)
    finally:
        c.close()


def test_host_pointer_batches_split(coder):
    """A host batch of >= 32768 packets and >= 32 MB runs in two halves on two
    contexts of the device (rc_host.c run_host_split: the second half's input
    DMA after the first's, the halves' kernels side by side): bit-exact
    against the oracle both ways, gapped compressed slots, and the hand-off
    counts of both halves reported together."""
    import ctypes as C
    from oracle.pyoracle import compress_batch as ocompress, fnv_digest
    d, o, l = synth.mixed_batch(50000, seed=17)          # ~36 MB: split
    assert d.size >= 32 << 20
    lib = coder.lib
    n = len(l)
    ln = l.astype(np.uint32)
    cap = (2 * ln.astype(np.int64) + 64).astype(np.uint32)
    coff = np.zeros(n, np.uint64)
    coff[1:] = np.cumsum(cap[:-1].astype(np.uint64) + 5)
    cout = np.zeros(int(coff[-1] + cap[-1]) + 16, np.uint8)
    clen = np.zeros(n, np.uint32)
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    assert lib.enet_rc_compress_batch_host(coder.ctx, p(d), p(o), p(ln), n, p(cout), p(coff), p(cap), p(clen)) == 0
    # the batch ran in pieces, the later ones on contexts configured like this one
    assert lib.enet_rc_last_split(coder.ctx) >= 2
    flags = lib.enet_rc_config_flags(coder.ctx)
    assert flags & 0x80000000 == 0, hex(flags)
    assert bool(flags & 2) == (coder.variant != "lane3-only") and bool(flags & 8) == (coder.variant != "lane3-only")
    assert bool(flags & 16) == (coder.variant == "enc2-slow")
    if getattr(coder, "variant", "") == "lane3":
        assert coder.last_lane_count() == 0 and coder.last_exact_count() == 0
    want, wo, wcap, wl = ocompress(d, o, l, "port")
    assert np.array_equal(clen, wl)
    assert fnv_digest(cout, coff, clen) == fnv_digest(want, wo, wl)
    dout = np.zeros(int(o[-1]) + int(l[-1]) + 16, np.uint8)
    dlen = np.zeros(n, np.uint32)
    assert lib.enet_rc_decompress_batch_host(coder.ctx, p(cout), p(coff), p(clen), n, p(dout), p(o), p(ln),
                                             p(dlen)) == 0
    assert lib.enet_rc_last_split(coder.ctx) >= 2
    if getattr(coder, "variant", "") == "lane3":
        assert coder.last_lane_count() == 0 and coder.last_exact_count() == 0
    assert np.array_equal(dlen, ln)
    assert np.array_equal(dout[: d.size], d)
    # game state: the fast decoder hands every packet of both halves on
    g, go, gl = synth.gamestate_batch(40000, 1200)
    gn = len(gl)
    gln = gl.astype(np.uint32)
    gcap = (2 * gln.astype(np.int64) + 64).astype(np.uint32)
    gcoff = np.zeros(gn, np.uint64)
    gcoff[1:] = np.cumsum(gcap[:-1].astype(np.uint64))
    gout = np.zeros(int(gcoff[-1] + gcap[-1]) + 16, np.uint8)
    glen = np.zeros(gn, np.uint32)
    assert lib.enet_rc_compress_batch_host(coder.ctx, p(g), p(go), p(gln), gn, p(gout), p(gcoff), p(gcap),
                                           p(glen)) == 0
    gback = np.zeros(g.size + 16, np.uint8)
    gblen = np.zeros(gn, np.uint32)
    assert lib.enet_rc_decompress_batch_host(coder.ctx, p(gout), p(gcoff), p(glen), gn, p(gback), p(go), p(gln),
                                             p(gblen)) == 0
    assert np.array_equal(gblen, gln) and np.array_equal(gback[: g.size], g)
    if getattr(coder, "variant", "") == "lane3":
        assert coder.last_lane_count() == gn


def test_host_pointer_batches_uniform_slots(coder):
    """Host batches whose compressed packets sit in slots at a uniform, odd
    pitch from an odd base (rc_host.c run_host: the strided H2D of max_len
    bytes per slot for the decompress input; the GPU scatter of the packed
    results into the caller's slots for the compress output): bit-exact
    against the oracle, the last slot's bytes beyond its packet untouched."""
    import ctypes as C
    from oracle.pyoracle import compress_batch as ocompress, fnv_digest
    d, o, l = synth.mixed_batch(26000, seed=91)          # > 16 MB each way
    lib = coder.lib
    n = len(l)
    ln = l.astype(np.uint32)
    pitch = 2 * 1392 + 64 + 1
    cap = np.full(n, pitch - 1, np.uint32)
    coff = (5 + np.arange(n, dtype=np.uint64) * np.uint64(pitch)).astype(np.uint64)
    cout = np.full(int(coff[-1]) + pitch + 64, 0xA5, np.uint8)
    clen = np.zeros(n, np.uint32)
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    assert lib.enet_rc_compress_batch_host(coder.ctx, p(d), p(o), p(ln), n, p(cout), p(coff), p(cap), p(clen)) == 0
    want, wo, wcap, wl = ocompress(d, o, l, "port")
    assert np.array_equal(clen, wl)
    assert fnv_digest(cout, coff, clen) == fnv_digest(want, wo, wl)
    assert np.all(cout[int(coff[-1]) + int(clen[-1]):] == 0xA5)
    dout = np.zeros(int(o[-1]) + int(l[-1]) + 16, np.uint8)
    dlen = np.zeros(n, np.uint32)
    assert lib.enet_rc_decompress_batch_host(coder.ctx, p(cout), p(coff), p(clen), n, p(dout), p(o), p(ln),
                                             p(dlen)) == 0
    assert np.array_equal(dlen, ln)
    assert np.array_equal(dout[: d.size], d)


def test_device_decoder_bounded_vs_oracle(coder):
    """enet_rc_decompress_batch_device_bounded: the caller's output bound sizes
    the wave decoder's model, so 513-1024-packet batches decode one wavefront
    per packet; bit-exact, including a bound below some caps (those packets
    outgrow the smaller model and take the exact path)."""
    from oracle.pyoracle import Coder
    port = Coder("port")
    rng = np.random.default_rng(91)
    for n, bound in ((513, 1400), (1000, 1400), (1280, 1200), (600, 200)):
        pk = [rng.integers(0, int(rng.choice([2, 17, 256])), size=int(rng.integers(1, 1401)),
                           dtype=np.uint8).tobytes() for _ in range(n)]
        caps = [2 * len(p) + 64 for p in pk]
        res = _run(coder, False, pk, caps)
        assert res == [port.compress(p, out_limit=c) for p, c in zip(pk, caps)]
        back = _run(coder, True, [r[1] for r in res], [len(p) for p in pk], max_out=bound)
        assert back == [(len(p), p) for p in pk], f"n={n} bound={bound}"


def test_host_pointer_decoder_sized_by_out_cap(coder):
    """Host-pointer decompress batches pass max(out_cap) down (rc_host.c
    run_host), so the wave decoder sizes its LDS arena by the output bound
    and batches of 513-1024 packets of <= 1400 B now fit on the chip at one
    wavefront per packet (rc_kernels.hip wave_lds).  Bit-exact against the
    oracle on both sides of the old 512-packet limit, with tight caps (a
    model outgrowing the smaller arena must take the exact path)."""
    import ctypes as C
    from oracle.pyoracle import Coder
    port = Coder("port")
    rng = np.random.default_rng(77)
    lib = coder.lib
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    for n in (513, 1000, 1280):
        pk = [rng.integers(0, int(rng.choice([2, 17, 256])), size=int(rng.integers(1, 1401)),
                           dtype=np.uint8).tobytes() for _ in range(n)]
        ln = np.array([len(x) for x in pk], np.uint32)
        o = np.zeros(n, np.uint64)
        o[1:] = np.cumsum(ln[:-1].astype(np.uint64))
        d = np.frombuffer(b"".join(pk), np.uint8).copy()
        cap = (2 * ln.astype(np.int64) + 64).astype(np.uint32)
        coff = np.zeros(n, np.uint64)
        coff[1:] = np.cumsum(cap[:-1].astype(np.uint64))
        cout = np.zeros(int(coff[-1] + cap[-1]) + 16, np.uint8)
        clen = np.zeros(n, np.uint32)
        assert lib.enet_rc_compress_batch_host(coder.ctx, p(d), p(o), p(ln), n, p(cout), p(coff), p(cap),
                                               p(clen)) == 0
        for i in range(n):
            got = cout[int(coff[i]): int(coff[i]) + int(clen[i])].tobytes()
            assert (int(clen[i]), got) == port.compress(pk[i], out_limit=int(cap[i])), f"n={n} packet {i}"
        dout = np.zeros(d.size + 16, np.uint8)
        dlen = np.zeros(n, np.uint32)
        assert lib.enet_rc_decompress_batch_host(coder.ctx, p(cout), p(coff), p(clen), n, p(dout), p(o), p(ln),
                                                 p(dlen)) == 0
        assert np.array_equal(dlen, ln), f"n={n}"
        assert np.array_equal(dout[: d.size], d), f"n={n}"


def test_long_packets_batch_vs_oracle(coder):
    """2048 packets of 1900-4096 B (random, low-entropy, runs): compress.c's
    model reset at 4094 nodes happens inside the lane kernels (rc_lane3.hip
    lane_reset); bit-exact against the oracle and back."""
    from oracle.pyoracle import compress_batch as ocompress, fnv_digest
    rng = np.random.default_rng(23)
    pk = []
    for i in range(2048):
        n = int(rng.integers(1900, 4097))
        k = i % 4
        if k == 0:
            p = rng.integers(0, 256, n, dtype=np.uint8)
        elif k == 1:
            p = rng.integers(0, 256, n, dtype=np.uint8) & np.uint8(rng.integers(1, 64))
        elif k == 2:
            p = (np.cumsum(rng.integers(-2, 3, n)) & 0xFF).astype(np.uint8)
        else:
            p = np.repeat(rng.integers(0, 256, n // 16 + 1, dtype=np.uint8), 16)[:n]
        pk.append(p.tobytes())
    d, o, l = _pack(pk)
    out, oo, cap, ol = ocompress(d, o, l, "port")
    res = _run(coder, False, pk, [int(c) for c in cap])
    gl = np.array([r[0] for r in res], np.uint32)
    assert np.array_equal(gl, ol)
    blob = np.frombuffer(b"".join(r[1] for r in res), np.uint8)
    goff = np.concatenate([[0], np.cumsum(gl[:-1].astype(np.uint64))]).astype(np.uint64)
    assert fnv_digest(blob, goff, gl) == fnv_digest(out, oo, ol)
    back = _run(coder, True, [r[1] for r in res], [len(p) for p in pk])
    assert all(b == (len(p), p) for b, p in zip(back, pk))


def test_device_decoder_small_bounds(coder):
    """Small output bounds (game-state-sized packets, bound 64, bound 1, and the
    largest bound 0xFFFFFFFF): the wave decoder's arena has a floor of 4 KB, so
    a small bound never routes valid streams to the 256-thread exact path
    (rc_kernels.hip arena_bytes_for).  Bit-exact, and no exact-path packets
    where every stream fits its model."""
    from oracle.pyoracle import Coder
    port = Coder("port")
    rng = np.random.default_rng(64)
    for n, lo, hi, bound in ((1024, 16, 65, 64), (256, 1, 2, 1), (300, 1, 400, 0xFFFFFFFF), (1024, 48, 49, 48)):
        pk = [rng.integers(0, int(rng.choice([2, 17, 256])), size=int(rng.integers(lo, hi)),
                           dtype=np.uint8).tobytes() for _ in range(n)]
        caps = [2 * len(p) + 64 for p in pk]
        res = _run(coder, False, pk, caps)
        assert res == [port.compress(p, out_limit=c) for p, c in zip(pk, caps)]
        back = _run(coder, True, [r[1] for r in res], [len(p) for p in pk], max_out=bound)
        assert back == [(len(p), p) for p in pk], f"n={n} bound={bound}"
        assert coder.last_exact_count() == 0, f"n={n} bound={bound}: valid streams took the exact path"


def test_small_packets_compress_not_exact(coder):
    """Compress batches of short packets (max_len < 94) stay on the fast
    kernels: the arena floor keeps them off the exact path."""
    from oracle.pyoracle import Coder
    port = Coder("port")
    rng = np.random.default_rng(48)
    pk = [rng.integers(0, 256, size=int(rng.integers(1, 65)), dtype=np.uint8).tobytes() for _ in range(1024)]
    caps = [2 * len(p) + 64 for p in pk]
    res = _run(coder, False, pk, caps)
    assert res == [port.compress(p, out_limit=c) for p, c in zip(pk, caps)]
    assert coder.last_exact_count() == 0


def test_host_batches_around_checksummed_datagrams(coder):
    """One context: a large host batch (device-side packing buffers), then a
    checksummed datagram encode with a larger n (grows the datagram scratch),
    then a large host batch again, all bit-exact.  Guards the ownership of the
    packing buffers (rc_host.c pack_reserve / dgram_reserve)."""
    import ctypes as C
    from oracle.pyoracle import compress_batch as ocompress, datagram_encode, fnv_digest, Coder
    lib = coder.lib
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    d, o, l = synth.mixed_batch(3000)            # > 1 MiB out: the packing path
    n = len(l)
    ln = l.astype(np.uint32)
    cap = (2 * ln.astype(np.int64) + 64).astype(np.uint32)
    coff = np.zeros(n, np.uint64)
    coff[1:] = np.cumsum(cap[:-1].astype(np.uint64))
    want, wo, wcap, wl = ocompress(d, o, l, "port")

    def host_round():
        cout = np.zeros(int(coff[-1] + cap[-1]) + 16, np.uint8)
        clen = np.zeros(n, np.uint32)
        assert lib.enet_rc_compress_batch_host(coder.ctx, p(d), p(o), p(ln), n, p(cout), p(coff), p(cap),
                                               p(clen)) == 0
        assert np.array_equal(clen, wl)
        assert fnv_digest(cout, coff, clen) == fnv_digest(want, wo, wl)

    host_round()
    port = Coder("port")
    rng = np.random.default_rng(3)
    dg = [b"\x80\x01\x00\x02" + bytes(4) + rng.integers(0, 3, size=int(rng.integers(1, 1200)),
                                                          dtype=np.uint8).tobytes() for _ in range(4000)]
    seeds = [int(s) for s in rng.integers(0, 2**32, size=len(dg))]
    enc = coder.datagrams(False, dg, checksum=True, seeds=seeds)
    for i in range(0, len(dg), 97):
        assert enc[i] == datagram_encode(dg[i], True, seeds[i], port)
    host_round()


_CHUNK_CASE = {}


def test_encoder_chunks_vs_oracle(coder):
    """More packets than one record-stream chunk: at max_len 1392 the 1-GB
    stream (rc_host.c ENC2_STREAM_MAX) holds ~96 Ki packet slots, rounded down
    to whole code-pass rounds (rc_enc2.hip rc_hip_enc2_launch), so 100000 ragged
    packets run as two chunks over the length-binned order.  Bit-exact against
    the oracle (batch digest), then the round trip."""
    from oracle.pyoracle import compress_batch as ocompress, fnv_digest
    if not _CHUNK_CASE:
        d, o, l = synth.mixed_batch(100000, seed=synth.SEED ^ 0x43484B53)
        out, oo, cap, ol = ocompress(d, o, l, "port")
        _CHUNK_CASE.update(d=d, o=o, l=l, cap=cap, digest=fnv_digest(out, oo, ol), total=int(ol.sum()))
    c = _CHUNK_CASE
    n = len(c["l"])
    din, doff, dlen = _dev(c["d"], torch.uint8), _dev(c["o"], torch.int64), _dev(c["l"], torch.int32)
    cap = _dev(c["cap"], torch.int32)
    coff = torch.zeros(n, dtype=torch.int64, device="cuda")
    coff[1:] = torch.cumsum(cap[:-1].to(torch.int64), 0)
    cout = torch.empty(int(coff[-1] + cap[-1]), dtype=torch.uint8, device="cuda")
    clen = torch.zeros(n, dtype=torch.int32, device="cuda")
    coder.compress_batch(din, doff, dlen, cout, coff, cap, clen, max_len=int(c["l"].max()))
    torch.cuda.synchronize()
    cl = clen.cpu().numpy().astype(np.uint32)
    assert int(cl.sum()) == c["total"]
    assert fnv_digest(cout.cpu().numpy(), coff.cpu().numpy().astype(np.uint64), cl) == c["digest"]
    dout = torch.empty_like(din)
    dl = torch.zeros(n, dtype=torch.int32, device="cuda")
    coder.decompress_batch(cout, coff, clen, dout, doff, dlen, dl, max_len=int(cl.max()))
    torch.cuda.synchronize()
    assert torch.equal(dl, dlen)
    assert torch.equal(dout, din)


def test_gather_batch_fixtures_and_oracle(coder):
    """enet_rc_compress_gather_batch_host: the reference's gather fixtures in
    one batch, then random gather lists (empty first buffers, empty later
    buffers -- the phantom byte, compress.c:275-284 -- and single spans)
    against the oracle's per-list compress."""
    from oracle.pyoracle import Coder
    cases = [c for c in golden_io.gather_cases() if c["in_limit"] > 0]
    backing, lists, caps = b"", [], []
    for c in cases:
        base = len(backing)
        backing += c["backing"]
        lists.append([(base + s, l) for s, l in c["spans"]])
        caps.append(c["out_limit"])
    res = coder.compress_gather_batch(backing, lists, caps)
    for c, r in zip(cases, res):
        assert r[0] == c["ret"], c["spans"][:4]
        if c["ret"]:
            assert r[1] == c["expect"]
    # random lists, enough bytes for the threaded flattening (> 16 MB)
    from oracle.pyoracle import compress_batch as ocompress
    rng = np.random.default_rng(17)
    backing = rng.integers(0, 8, size=1 << 20, dtype=np.uint8).tobytes()
    lists, flat = [], []
    for i in range(24000):
        spans = []
        for j in range(int(rng.integers(1, 6))):
            ln = 0 if rng.random() < 0.2 else int(rng.integers(1, 800))
            spans.append((int(rng.integers(0, len(backing) - 1024)), ln))
        lists.append(spans)
        # compress.c:275-284: the first buffer as is, a later empty one its data[0]
        f = backing[spans[0][0]: spans[0][0] + spans[0][1]]
        for s0, l0 in spans[1:]:
            f += backing[s0: s0 + l0] if l0 else backing[s0: s0 + 1]
        flat.append(f)
    keep = [i for i, f in enumerate(flat) if f]
    d, o, l = synth.pack([flat[i] for i in keep])
    ref, roff, cap, rlen = ocompress(d, o, l, "port")
    caps = [2 * len(f) + 64 for f in flat]
    res = coder.compress_gather_batch(backing, lists, caps)
    assert sum(len(f) for f in flat) > (16 << 20)
    for j, i in enumerate(keep):
        assert res[i][0] == int(rlen[j])
        assert res[i][1] == ref[int(roff[j]): int(roff[j]) + int(rlen[j])].tobytes()
    assert all(res[i] == (0, b"") for i, f in enumerate(flat) if not f)
