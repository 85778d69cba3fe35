"""The bucket-history decoder model (tests/proto/histdec.py, restating
rc_dec4.hip's algebra) against the oracle and the golden fixtures, on the
CPU: valid streams at every output limit edge and corrupt streams decode to
the reference's return value and bytes, or are handed to the lane kernels
(None) where the GPU decoder would."""
import numpy as np

from enet_amd import synth
from tests import golden_io
from tests.proto import histdec


def test_golden_decompress_fixtures():
    n_fast = 0
    for c in golden_io.decompress_cases():
        r = histdec.decode(c["input"], c["out_limit"])
        if r is None:
            continue
        n_fast += 1
        assert r[0] == c["ret"]
        if c["ret"]:
            assert r[1] == c["expect"]
    assert n_fast > 1000


def test_random_packets_and_limits():
    from oracle.pyoracle import Coder
    port = Coder("port")
    d, o, l = synth.random_batch(12, 1200)
    rng = np.random.default_rng(4)
    pk = [d[int(o[i]): int(o[i]) + 1200].tobytes() for i in range(12)]
    pk += [rng.integers(0, 256, size=int(rng.integers(1, 1920)), dtype=np.uint8).tobytes() for _ in range(12)]
    fast = 0
    for p in pk:
        c = port.compress(p)[1]
        for lim in (len(p), len(p) - 1, 4096):
            r = histdec.decode(c, lim)
            if r is not None:
                fast += 1
                assert r == port.decompress(c, lim)
    assert fast >= 60


def test_bails_where_the_lanes_take_over():
    from oracle.pyoracle import Coder
    port = Coder("port")
    c = port.compress(bytes(300))[1]                  # one bucket of 299 positions
    assert histdec.decode(c, 4096) is None
    c = port.compress(synth.de_bruijn_bytes(2100))[1]  # model reset at 4094 nodes
    assert histdec.decode(c, 4096) is None
