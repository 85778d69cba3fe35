"""The CPU oracle (oracle/rc_oracle.c) against fixtures made by the real compress.c.

This pins the oracle before anything else is compared with it (task rule ③)."""
import numpy as np
import pytest

from enet_amd import synth
from oracle.pyoracle import Coder, compress_batch, decompress_batch, fnv_digest, have_reference
from tests import golden_io


@pytest.fixture(scope="module")
def port():
    c = Coder("port")
    yield c
    c.close()


def test_kats(port):
    # SURVEY.md §8c known answers (measured on the reference)
    assert port.compress(b"\x5a") == (4, bytes.fromhex("5aa55aa5"))
    assert port.compress(b"hello world") == (13, bytes.fromhex("68fbe0c33d70a617f8bc911698"))
    assert port.compress(b"\0" * 1200) == (9, bytes.fromhex("0103e861fe44689a30"))


def test_compress_fixtures(port):
    cases = golden_io.compress_cases()
    assert len(cases) > 200
    for c in cases:
        r, out = port.compress(c["input"], out_limit=c["out_limit"], in_limit=c["in_limit"])
        assert r == c["ret"], (len(c["input"]), c["out_limit"])
        assert out == c["expect"]


def test_gather_fixtures(port):
    for c in golden_io.gather_cases():
        r, out = port.compress_gather(c["backing"], c["spans"], c["in_limit"], c["out_limit"])
        assert (r, out) == (c["ret"], c["expect"]), c["spans"][:4]


def test_decompress_fixtures(port):
    cases = golden_io.decompress_cases()
    assert len(cases) > 3000
    nonzero_garbage = 0
    for c in cases:
        r, out = port.decompress(c["input"], c["out_limit"])
        assert r == c["ret"]
        assert out == c["expect"]
        nonzero_garbage += r > 0
    assert nonzero_garbage > 100


def test_c1_digest():
    d, o, l = synth.random_batch(4096, 256)
    g = golden_io.digests()["C1_random_4096x256"]
    assert fnv_digest(d, o, l) == g["input_fnv"]
    out, oo, cap, ol = compress_batch(d, o, l, "port")
    assert int(ol.sum()) == g["out_bytes"]
    assert fnv_digest(out, oo, ol) == g["digest"]
    dec, do, dl = decompress_batch(out, oo, ol, l)
    assert np.array_equal(dl, l)
    assert fnv_digest(dec, do, dl) == g["input_fnv"]


def test_synth_inputs_pinned():
    g = golden_io.digests()
    d, o, l = synth.gamestate_batch(65536, 1200)
    assert fnv_digest(d, o, l) == g["C3_gamestate_65536x1200"]["input_fnv"]
    d, o, l = synth.random_batch(65536, 1200)
    assert fnv_digest(d, o, l) == g["C2_random_65536x1200"]["input_fnv"]


@pytest.mark.skipif(not have_reference(), reason="reference build (oracle/_ref) absent")
def test_port_matches_reference_fuzz(port):
    ref = Coder("reference")
    rng = np.random.default_rng(7)
    for t in range(300):
        n = int(rng.integers(1, 2000))
        alpha = int(rng.choice([2, 5, 17, 256]))
        data = (rng.integers(0, alpha, size=n)).astype(np.uint8).tobytes()
        lim = int(rng.choice([n, 2 * n + 64, n // 2 + 1]))
        assert port.compress(data, out_limit=lim) == ref.compress(data, out_limit=lim)
        g = rng.integers(0, 256, size=int(rng.integers(1, 64)), dtype=np.uint8).tobytes()
        assert port.decompress(g, 2048) == ref.decompress(g, 2048)


def test_cpu_bench_port_roundtrip():
    d, o, l = synth.random_batch(256, 1200)
    r = __import__("oracle.pyoracle", fromlist=["cpu_roundtrip"]).cpu_roundtrip(d, o, l, 2, kind="port")
    assert r["mismatches"] == 0 and r["compressed_bytes"] > 256 * 1200
