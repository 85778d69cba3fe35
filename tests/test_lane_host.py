"""Host (CPU) build of the lane kernels' per-lane logic (enet_amd/csrc/rc_lane3.hip,
and the record-light decoder rc_dec6.hip in front of it, compiled with
tests/proto/lane_host_shim.h) against the reference fixtures.

The lane kernel is scalar code per lane, so its model and coder logic can be
exercised here without a GPU; the -m gpu tests then check the real kernel."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from tests import golden_io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tests", "proto", "liblanehost.so")


# v3: the lane kernels alone;
# v6: the record-light decoder (rc_dec6.hip) and its check in front of them, loading its own input;
# v6s: rc_dec6.hip with its input through the LDS slot (rc_slot.h; the helper run after every
# step), as on the GPU
@pytest.fixture(scope="module", params=["v3", "v6", "v6s"])
def lane(request):
    so = SO.replace("liblanehost", "liblanehost" + request.param[1:])
    csrc = os.path.join(ROOT, "enet_amd", "csrc")
    src = [os.path.join(ROOT, "tests", "proto", "lane_host.cpp")] + \
        [os.path.join(csrc, f) for f in ("rc_lane3.hip", "rc_dec6.hip", "rc_dec6_rare.h",
                                         "rc_slot.h", "rc_lane_common.h", "rc_root3.h")]
    if not os.path.exists(so) or os.path.getmtime(so) < max(os.path.getmtime(s) for s in src):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared"] +
                              {"v3": [], "v6": ["-DDEC6"], "v6s": ["-DDEC6", "-DDEC6S"]}[request.param] +
                              ["-I", csrc, "-I", os.path.join(ROOT, "tests", "proto"), "-o", so, src[0]])
    lib = C.CDLL(so)
    lib.lane_host_run.argtypes = [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32,
                                  C.POINTER(C.c_uint32)]
    ol = C.c_uint32()

    def run(dec, data, cap, max_len=None):
        a = np.frombuffer(bytes(data) + b"\0" * 16, dtype=np.uint8).copy()
        out = np.zeros(max(cap, 1) + 16, np.uint8)
        ml = max_len or max(len(data), 16)
        rc = lib.lane_host_run(dec, a.ctypes.data, len(data), out.ctypes.data, cap, ml, C.byref(ol))
        run.left += rc == 2
        if rc == 1:
            return "exact", b""
        return ol.value, out[: ol.value].tobytes()
    run.version = request.param
    run.lib = lib
    run.left = 0
    return run


def test_lane_logic_compress_fixtures(lane):
    for c in golden_io.compress_cases():
        if c["in_limit"] != len(c["input"]):
            continue
        r = lane(0, c["input"], c["out_limit"])
        if r[0] == "exact":      # (allowed only for packets long enough to reach the model reset)
            assert len(c["input"]) > 1919
            continue
        assert r[0] == c["ret"], (len(c["input"]), c["out_limit"])
        if c["ret"]:
            assert r[1] == c["expect"]


def test_lane_logic_decompress_fixtures(lane):
    exact = 0
    lane.left = 0
    cases = golden_io.decompress_cases()
    for c in cases:
        r = lane(1, c["input"], c["out_limit"])
        if r[0] == "exact":      # corrupt stream pointing past symbol 255: exact path
            exact += 1
            assert c["ret"] >= 0
            continue
        assert r[0] == c["ret"]
        if c["ret"]:
            assert r[1] == c["expect"]
    assert 0 < exact < 2000
    if lane.version in ("v6", "v6s"):     # most fixtures are garbage or low-entropy: those are left to the lanes
        assert 0 < lane.left < len(cases) - 1000, (lane.left, len(cases))


def test_dec6_takes_random_packets(lane):
    """The record-light decoder decodes random packets up to MTU size itself
    (no bucket reaches its limits) and matches the oracle at every output
    limit edge."""
    if lane.version == "v3":
        pytest.skip("dec6 only")
    from oracle.pyoracle import Coder
    port = Coder("port")
    rng = np.random.default_rng(11)
    lane.left = 0
    for n in list(rng.integers(1, 1393, size=40)) + [1200] * 8 + [1, 2, 3, 1392]:
        p = rng.integers(0, 256, size=int(n), dtype=np.uint8).tobytes()
        r, c = port.compress(p, 2 * len(p) + 64)
        for lim in (len(p), len(p) - 1, 4096):
            got = lane(1, c, lim)
            assert got == port.decompress(c, lim), (n, lim)
    assert lane.left == 0


def test_dec6_model_reset(lane):
    """The record-light decoder through compress.c's model reset (4094 nodes,
    compress.c:148-157): random packets of 1900-4096 bytes (one or two resets)
    decoded by dec6 itself, checked per model segment, against the oracle at
    output limits on either side of a reset; corrupt streams stay correct."""
    if lane.version not in ("v6", "v6s"):
        pytest.skip("dec6 only")
    from oracle.pyoracle import Coder
    port = Coder("port")
    rng = np.random.default_rng(29)
    valid_left = 0
    sizes = [1900, 1950, 2100, 2731, 3000, 4095, 4096] + list(rng.integers(1920, 4097, size=8))
    for n in sizes:
        p = rng.integers(0, 256, size=int(n), dtype=np.uint8).tobytes()
        r, c = port.compress(p, 2 * len(p) + 64)
        lane.left = 0
        for lim in (len(p), len(p) - 1, 2000, 4096):
            got = lane(1, c, lim, max_len=4096)
            assert got == port.decompress(c, lim), (n, lim)
        valid_left += lane.left
        bad = bytearray(c)
        bad[len(bad) * 3 // 4] ^= 0x21
        got = lane(1, bytes(bad), 4096, max_len=4096)
        if got[0] != "exact":
            assert got == port.decompress(bytes(bad), 4096)
    assert valid_left == 0, valid_left


def test_dec6_bucket_capacity(lane):
    """A bucket of 25-28 order-1 elements fills the record-light decoder's
    second record (elements 8-27, rc_dec6_rare.h kTabCap): the decoder keeps
    the packet; past 28 it leaves it to the lane kernels.  Against the oracle."""
    if lane.version not in ("v6", "v6s"):
        pytest.skip("dec6 only")
    from oracle.pyoracle import Coder
    port = Coder("port")
    rng = np.random.default_rng(31)
    for k in (20, 25, 27, 28, 29, 31):
        x = rng.integers(8, 256, size=1200, dtype=np.uint8)
        at = rng.choice(np.arange(2, 1199), size=k, replace=False)
        x[at] = 7                                  # bucket 7: the k bytes after them
        p = x.tobytes()
        r, c = port.compress(p, 2 * len(p) + 64)
        lane.left = 0
        assert lane(1, c, len(p)) == port.decompress(c, len(p)), k
        if k <= 27:                                # (an adjacent pair of 7s can add an element)
            assert lane.left == 0, k


def test_lane_logic_region_overflow_routes_exact(lane):
    # a tiny region (max_len hint 16) cannot hold a 1200-byte random packet's model
    # (v3 keeps single-symbol order-2 contexts inline, so it needs a small
    # alphabet -- many order-2 contexts with several symbols -- to fill its arena)
    data = np.random.default_rng(3).integers(0, 256, 1200, dtype=np.uint8)
    data &= 15
    assert lane(0, data.tobytes(), 4096, max_len=16)[0] == "exact"


def test_lane_logic_dense_order2_contexts(lane):
    """Packets whose order-2 contexts go dense (more than 24 symbols): game
    state ((0, 0) in every packet -- the lane's LDS dense block), several dense
    order-2 contexts per packet (the first in the LDS block, the others in the
    arena), long packets across the model reset.  Both directions, against
    the oracle."""
    from enet_amd import synth
    from oracle.pyoracle import Coder
    port = Coder("port")
    rng = np.random.default_rng(23)
    d, o, l = synth.gamestate_batch(6, 1200)
    pk = [d[int(o[i]): int(o[i]) + 1200].tobytes() for i in range(6)]
    for n in (1500, 3000, 4096):
        # three heavy contexts: bytes after (0, 0), (1, 1) and (2, 2) drawn from 40 values
        x = np.zeros(n, np.uint8)
        for j in range(2, n):
            x[j] = rng.integers(0, 40) if x[j - 1] == x[j - 2] and rng.random() < 0.5 else x[j - 1]
        pk.append(x.tobytes())
        pk.append(np.where(rng.random(n) < 0.7, 0, rng.integers(0, 256, n)).astype(np.uint8).tobytes())
    for p in pk:
        cap = 2 * len(p) + 64
        ref = port.compress(p, out_limit=cap)
        assert lane(0, p, cap, max_len=len(p)) == ref
        assert lane(1, ref[1], len(p), max_len=len(p)) == (len(p), p)


def _injection_lib(extra, tag):
    csrc = os.path.join(ROOT, "enet_amd", "csrc")
    so = os.path.join(ROOT, "tests", "proto", f"liblanehost6s_{tag}.so")
    src = [os.path.join(ROOT, "tests", "proto", "lane_host.cpp")] + \
        [os.path.join(csrc, f) for f in ("rc_dec6.hip", "rc_dec6_rare.h", "rc_slot.h", "rc_lane_common.h")]
    if not os.path.exists(so) or os.path.getmtime(so) < max(os.path.getmtime(s) for s in src):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-DDEC6", "-DDEC6S"] + extra +
                              ["-I", csrc, "-I", os.path.join(ROOT, "tests", "proto"), "-o", so, src[0]])
    lib = C.CDLL(so)
    lib.lane_host_run.argtypes = [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32,
                                  C.POINTER(C.c_uint32)]
    return lib


def _inject_run(lib, packets):
    """Each packet decoded once per injection kind with one chunk it takes from
    its slot replaced (tests/proto/lane_host.cpp slot_host_taken: the chunk
    before it -- the slot's stale content --, the one after it, or zeros);
    returns (decodes, results that differ from the packet)."""
    ol = C.c_uint32()
    rng = np.random.default_rng(41)
    total = wrong = 0
    for p, c in packets:
        a = np.frombuffer(c + b"\0" * 16, np.uint8).copy()
        for kind in (0, 1, 2):
            out = np.zeros(len(p) + 16, np.uint8)
            lib.lane_host_inject(-1, 0)
            lib.lane_host_run(1, a.ctypes.data, len(c), out.ctypes.data, len(p), 1400, C.byref(ol))
            takes = lib.lane_host_inject(-1, 0)
            if takes == 0:
                continue
            lib.lane_host_inject(int(rng.integers(0, takes)), kind)
            out = np.zeros(len(p) + 16, np.uint8)
            rc = lib.lane_host_run(1, a.ctypes.data, len(c), out.ctypes.data, len(p), 1400, C.byref(ol))
            lib.lane_host_inject(-1, 0)
            total += 1
            if rc == 1 or (ol.value, out[: ol.value].tobytes()) != (len(p), p):
                wrong += rc != 1            # (rc 1: the exact path, which reads the true stream)
    return total, wrong


def test_dec6s_stale_chunk_injection():
    """A stale input chunk in the record-light decoder's slot (the r5a-type
    failure mode: a wrong length with a success code).  The decode of other
    bytes is a faithful decode of those bytes, so the bigram count alone lets
    some of them through; the hand-off's check sums (rc_slot.h slot_mix,
    compared by rc_dec6_verify) send every one to the lane kernels, which
    decode the true stream."""
    from oracle.pyoracle import Coder
    port = Coder("port")
    rng = np.random.default_rng(43)
    packets = []
    for _ in range(150):
        n = int(rng.integers(100, 1400))
        p = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        packets.append((p, port.compress(p, 2 * n + 64)[1]))
    total, wrong = _inject_run(_injection_lib([], "cks"), packets)
    assert total > 400 and wrong == 0, (total, wrong)
    total0, wrong0 = _inject_run(_injection_lib(["-DSLOT_NO_CKS", "-DDEC6_NO_USED_CHECK"], "nocks"), packets)
    assert total0 == total and wrong0 > 0, (total0, wrong0)   # the bigram count alone misses some
