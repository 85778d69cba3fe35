"""enet_crc32 (packet.c:143-163) -- SURVEY.md §8f row 2.

CPU: the oracle against the fixtures made by the reference's own enet_crc32
(tests/golden/crc_cases.npz) and against zlib.
GPU: the batch kernel (rc_crc32.hip) through the C ABI against the fixtures
and the oracle, with packets at unaligned offsets, every length 0..80, and
the full C2 batch; the per-datagram checksum callback on gather lists.
"""
import ctypes as C
import zlib

import numpy as np
import pytest

from enet_amd import synth
from tests import golden_io


def _net(v):
    """zlib's CRC -> the reference's return value (ENET_HOST_TO_NET_32 of it)."""
    return int.from_bytes(v.to_bytes(4, "big"), "little")


def test_oracle_crc_matches_reference_fixtures():
    from oracle.pyoracle import crc32_batch
    cases = golden_io.crc_cases()
    assert cases[0] == (b"123456789", _net(0xCBF43926))          # the CRC-32/IEEE check value
    blob = np.frombuffer(b"".join(c[0] for c in cases), np.uint8)
    ln = np.array([len(c[0]) for c in cases], np.uint32)
    off = np.concatenate([[0], np.cumsum(ln[:-1], dtype=np.uint64)]).astype(np.uint64)
    got = crc32_batch(blob if blob.size else np.zeros(1, np.uint8), off, ln, "port")
    assert [int(x) for x in got] == [c[1] for c in cases]


def test_oracle_crc_matches_zlib_mixed():
    from oracle.pyoracle import crc32_batch
    d, o, l = synth.mixed_batch(3000, lo=0, hi=4096, seed=21)
    got = crc32_batch(d, o, l, "port")
    for i in range(0, len(l), 7):
        assert int(got[i]) == _net(zlib.crc32(d[int(o[i]): int(o[i]) + int(l[i])].tobytes()))


# ----------------------------------------------------------------------- GPU
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def coder():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from enet_amd import RangeCoder
    c = RangeCoder()
    yield c
    c.close()


def _scatter_unaligned(packets, seed=0):
    """Packs packets at random byte offsets (gaps of 0..37 garbage bytes)."""
    rng = np.random.default_rng(seed)
    parts, offs, pos = [], [], 0
    for p in packets:
        gap = int(rng.integers(0, 38))
        parts.append(rng.integers(0, 256, gap, dtype=np.uint8).tobytes())
        pos += gap
        offs.append(pos)
        parts.append(p)
        pos += len(p)
    parts.append(rng.integers(0, 256, 64, dtype=np.uint8).tobytes())
    blob = np.frombuffer(b"".join(parts), np.uint8)
    return blob, np.array(offs, np.int64), np.array([len(p) for p in packets], np.int32)


def _gpu_crc(coder, blob, off, ln):
    din = torch.from_numpy(blob.copy()).cuda()
    res = coder.crc32_batch(din, torch.from_numpy(off).cuda(), torch.from_numpy(ln).cuda())
    torch.cuda.synchronize()
    return res.cpu().numpy().view(np.uint32)


@pytest.mark.gpu
def test_gpu_crc_fixtures_unaligned(coder):
    cases = golden_io.crc_cases()
    for seed in range(3):
        blob, off, ln = _scatter_unaligned([c[0] for c in cases], seed)
        got = _gpu_crc(coder, blob, off, ln)
        bad = [(len(c[0]), int(g), c[1]) for c, g in zip(cases, got) if int(g) != c[1]]
        assert not bad, bad[:8]


@pytest.mark.gpu
def test_gpu_crc_mixed_vs_oracle(coder):
    from oracle.pyoracle import crc32_batch
    d, o, l = synth.mixed_batch(1 << 15, lo=0, hi=4096, seed=8)
    got = _gpu_crc(coder, d, o.astype(np.int64), l.astype(np.int32))
    assert np.array_equal(got, crc32_batch(d, o, l, "port"))


@pytest.mark.gpu
def test_gpu_crc_c2_full_size(coder):
    from oracle.pyoracle import crc32_batch
    d, o, l = synth.random_batch(65536, 1200)
    got = _gpu_crc(coder, d, o.astype(np.int64), l.astype(np.int32))
    assert np.array_equal(got, crc32_batch(d, o, l, "port"))


@pytest.mark.gpu
def test_gpu_crc_host_and_callback(coder):
    from enet_amd._lib import ENetBuffer, get_lib
    lib = get_lib()
    for n in (0, 1, 3, 4, 5, 100, 1392, 4096):
        data = synth.random_bytes(n, n).tobytes()
        assert coder.crc32(data) == _net(zlib.crc32(data))
    # ENetChecksumCallback over a gather list == CRC of the concatenation
    pieces = [b"\x01\x02", b"", synth.random_bytes(1000, 3).tobytes(), b"xyz"]
    keep = [C.create_string_buffer(p, max(1, len(p))) for p in pieces]
    bufs = (ENetBuffer * len(pieces))()
    for i, (p, k) in enumerate(zip(pieces, keep)):
        bufs[i].data = C.addressof(k)
        bufs[i].dataLength = len(p)
    assert lib.enet_rc_crc32(bufs, len(pieces)) == _net(zlib.crc32(b"".join(pieces)))
