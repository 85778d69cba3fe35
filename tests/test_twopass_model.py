"""The two-pass decomposition of compress.c (tests/proto/twopass.py, the
Python model of rc_enc2.hip's record format) against the oracle and the
reference's golden fixtures, on the CPU.

This pins the algebra the HIP encoder relies on: order-1/order-2 coding
intervals are functions of the packet's own bytes (bucketed by the previous
byte), and a root-only model plus a range coder over those records
reproduces compress.c bit for bit.  Packets outside the fast path (a bucket
over 64 positions, >= 1920 bytes) must be reported as such (None).
"""
import numpy as np
import pytest

from enet_amd import synth
from tests import golden_io
from tests.proto import twopass


@pytest.fixture(scope="module")
def port():
    from oracle.pyoracle import Coder
    return Coder("port")


def test_golden_compress_fixtures():
    n_fast = 0
    for c in golden_io.compress_cases():
        if c["in_limit"] != len(c["input"]):
            continue
        r = twopass.compress(c["input"], c["out_limit"])
        if r is None:
            continue
        n_fast += 1
        assert r[0] == c["ret"], (len(c["input"]), c["out_limit"])
        if c["ret"]:
            assert r[1] == c["expect"]
    assert n_fast > 100


def test_random_and_mixed_packets(port):
    rng = np.random.default_rng(2)
    d, o, l = synth.random_batch(24, 1200)
    pk = [d[int(o[i]): int(o[i]) + 1200].tobytes() for i in range(24)]
    pk += [rng.integers(0, 256, size=int(rng.integers(1, 1920)), dtype=np.uint8).tobytes() for _ in range(40)]
    pk += [rng.integers(0, a, size=int(rng.integers(1, 400)), dtype=np.uint8).tobytes()
           for a in (7, 16, 40, 100) for _ in range(10)]
    fast = 0
    for p in pk:
        for lim in (2 * len(p) + 64, len(p)):
            r = twopass.compress(p, lim)
            if r is None:
                continue
            fast += 1
            assert r == port.compress(p, out_limit=lim)
    assert fast > 100


def test_gamestate_prefixes(port):
    d, o, l = synth.gamestate_batch(8, 1200)
    fast = 0
    for i in range(8):
        for n in (24, 100, 240, 600, 1200):
            p = d[int(o[i]): int(o[i]) + n].tobytes()
            r = twopass.compress(p, 2 * n + 64)
            if r is not None:
                fast += 1
                assert r == port.compress(p, out_limit=2 * n + 64)
    assert fast > 10


def test_fast_path_limits():
    assert twopass.scan(b"") is None
    assert twopass.scan(bytes(1920)) is None                  # long: possible model reset
    assert twopass.scan(bytes(66)) is None                    # 65 positions after a 0 byte
    assert twopass.scan(bytes(65)) is not None                # 64: still fast
    rnd = synth.random_bytes(1919, 7).tobytes()
    assert twopass.scan(rnd) is not None


# ---- wide mode (rc_enc2_wscan / rc_enc2_wcode): packets with big buckets,
# rescales included

def _wide_packets():
    rng = np.random.default_rng(5)
    d, o, l = synth.gamestate_batch(6, 1200)
    pk = [d[int(o[i]): int(o[i]) + 1200].tobytes() for i in range(6)]
    pk += [bytes(n) for n in (1, 2, 3, 100, 300, 1000, 1919)]           # one context, rescales
    pk += [bytes([7]) * n for n in (257, 1000)]
    pk += [rng.choice([0, 0, 0, 1, 2], size=n).astype(np.uint8).tobytes() for n in (200, 800, 1919)]
    pk += [(np.arange(n) % 2).astype(np.uint8).tobytes() for n in (500, 1919)]
    pk += [np.where(rng.random(n) < 0.8, 0, rng.integers(0, 256, n)).astype(np.uint8).tobytes() for n in (400, 1919)]
    pk += [rng.integers(0, 256, size=n, dtype=np.uint8).tobytes() for n in (1, 5, 300)]
    return pk


@pytest.mark.parametrize("dense_min,max_bucket", [(32, 64), (0, 64), (0, 0), (1000, 0)])
def test_wide_model_vs_oracle(port, monkeypatch, dense_min, max_bucket):
    """Default thresholds, dense walks for every big-bucket run, the big-bucket
    path for every bucket; (1000, 0): closed form everywhere, which must be
    exact on exactly the packets with no rescale."""
    monkeypatch.setattr(twopass, "DENSE_MIN", dense_min)
    monkeypatch.setattr(twopass, "MAX_BUCKET", max_bucket)
    closed_only = dense_min >= 1000
    n_ok = 0
    for p in _wide_packets():
        for lim in (2 * len(p) + 64, len(p)):
            r = twopass.compress_wide(p, lim)
            ref = port.compress(p, out_limit=lim)
            if closed_only:
                n_ok += r == ref
                continue
            assert r == ref, (len(p), lim)
    if closed_only:
        assert 0 < n_ok < 2 * len(_wide_packets())       # rescales exist in the set


def test_wide_model_golden_fixtures():
    n = 0
    for c in golden_io.compress_cases():
        if c["in_limit"] != len(c["input"]) or not 0 < len(c["input"]) <= twopass.MAX_LEN:
            continue
        r = twopass.compress_wide(c["input"], c["out_limit"])
        assert r[0] == c["ret"]
        if c["ret"]:
            assert r[1] == c["expect"]
        n += 1
    assert n > 100


def test_wide_model_long_packets_with_resets(port):
    """Packets of 1920-4096 B: model resets (compress.c:148-157) where the
    segment's node count reaches 4094; each segment is modelled afresh."""
    rng = np.random.default_rng(9)
    resets = 0
    for n in (1920, 2600, 4096):
        for p in (rng.integers(0, 256, n, dtype=np.uint8).tobytes(),
                  np.where(rng.random(n) < 0.6, 0, rng.integers(0, 256, n)).astype(np.uint8).tobytes(),
                  rng.integers(0, 40, n, dtype=np.uint8).tobytes(), bytes(n)):
            resets += sum(r[3] for r in twopass.scan_wide(p, 4096))
            for lim in (2 * n + 64, n):
                assert twopass.compress_wide(p, lim, 4096) == port.compress(p, out_limit=lim)
    assert resets >= 3
