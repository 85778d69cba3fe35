"""Synthetic packet batches for the range-coder benchmarks.

All generators are deterministic functions of a seed and are built on
splitmix64 so that the byte streams do not depend on numpy's RNG versions.
A batch is returned as ``(data, offsets, lengths)``: ``data`` is one packed
``uint8`` array and packet ``i`` is ``data[offsets[i] : offsets[i] + lengths[i]]``.

Configs (BASELINE.json ``configs``):
  C1  4096 x 256 B   random bytes            -> ``random_batch(4096, 256)``
  C2  65536 x 1200 B random bytes            -> ``random_batch(65536, 1200)``
  C3  65536 x 1200 B game-state records      -> ``gamestate_batch(65536, 1200)``
  C4  1 Mi packets of 64..1392 B random bytes -> ``mixed_batch(1 << 20)``
  C5  8 x C2 with distinct seeds             -> ``random_batch(65536, 1200, seed=SEED + rank)``
"""
from __future__ import annotations

import numpy as np

SEED = 0x454E4554  # "ENET"
_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, count: int, start: int = 0) -> np.ndarray:
    """Outputs ``start .. start+count-1`` of the splitmix64 stream of ``seed``."""
    with np.errstate(over="ignore"):
        idx = np.arange(start + 1, start + count + 1, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + idx * _GAMMA
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def random_bytes(nbytes: int, seed: int = SEED) -> np.ndarray:
    """Little-endian bytes of successive splitmix64 outputs."""
    words = splitmix64(seed, (nbytes + 7) // 8)
    return words.view(np.uint8)[:nbytes].copy()


def _uniform_offsets(n: int, size: int):
    off = np.arange(n, dtype=np.uint64) * np.uint64(size)
    ln = np.full(n, size, dtype=np.uint32)
    return off, ln


def random_batch(n: int, size: int, seed: int = SEED):
    """``n`` packets of ``size`` uniform-random bytes (packet i = bytes [i*size, (i+1)*size))."""
    data = random_bytes(n * size, seed)
    off, ln = _uniform_offsets(n, size)
    return data, off, ln


def gamestate_batch(n: int, size: int, seed: int = SEED ^ 0x47414D45):
    """Low-entropy packets made of 24-byte entity records (config C3).

    Record layout (little endian)::

        [0]     entity id, increments per record (wraps), random start per packet
        [1]     record type = 1
        [2:8]   x, y, z as u16; each starts at a random base per packet and
                random-walks by U[-3, 3] from record to record
        [8]     state U[0, 3]
        [9]     flags: a random byte with probability 1/16, else 0
        [10:12] 0, 0
        [12]    health = 100
        [13]    U[0, 2]
        [14:24] zeros
    A packet holds ``size // 24`` records; a ragged tail is zero-filled.
    """
    rec = size // 24
    r = splitmix64(seed, n * rec * 4 + n * 4)
    per_rec = r[: n * rec * 4].reshape(n, rec, 4)
    per_pkt = r[n * rec * 4:].reshape(n, 4)
    out = np.zeros((n, size), dtype=np.uint8)
    if rec:
        recs = out[:, : rec * 24].reshape(n, rec, 24)
        start_id = (per_pkt[:, 0] & np.uint64(0xFF)).astype(np.int64)
        recs[:, :, 0] = ((start_id[:, None] + np.arange(rec)[None, :]) & 0xFF).astype(np.uint8)
        recs[:, :, 1] = 1
        for axis in range(3):
            base = ((per_pkt[:, 1 + axis] >> np.uint64(7)) & np.uint64(0xFFFF)).astype(np.int64)
            step = ((per_rec[:, :, axis] % np.uint64(7)).astype(np.int64) - 3)
            pos = (base[:, None] + np.cumsum(step, axis=1)) & 0xFFFF
            recs[:, :, 2 + 2 * axis] = (pos & 0xFF).astype(np.uint8)
            recs[:, :, 3 + 2 * axis] = (pos >> 8).astype(np.uint8)
        w = per_rec[:, :, 3]
        recs[:, :, 8] = (w & np.uint64(3)).astype(np.uint8)
        flag_on = ((w >> np.uint64(8)) & np.uint64(15)) == 0
        recs[:, :, 9] = np.where(flag_on, ((w >> np.uint64(16)) & np.uint64(0xFF)), 0).astype(np.uint8)
        recs[:, :, 12] = 100
        recs[:, :, 13] = ((w >> np.uint64(24)) % np.uint64(3)).astype(np.uint8)
    data = out.reshape(-1)
    off, ln = _uniform_offsets(n, size)
    return data, off, ln


def mixed_batch(n: int, lo: int = 64, hi: int = 1392, seed: int = SEED ^ 0x4D495845):
    """``n`` packets with N = lo + U[0, hi-lo] random bytes (config C4, MTU-bounded)."""
    span = hi - lo + 1
    ln = (lo + (splitmix64(seed, n) % np.uint64(span))).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    if n > 1:
        off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    data = random_bytes(int(ln.sum(dtype=np.uint64)), seed ^ 0x5A5A5A5A)
    return data, off, ln


def pack(packets) -> tuple:
    """Packs a list of byte strings into ``(data, offsets, lengths)``."""
    ln = np.array([len(p) for p in packets], dtype=np.uint32)
    off = np.zeros(len(packets), dtype=np.uint64)
    if len(packets) > 1:
        off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    data = np.frombuffer(b"".join(bytes(p) for p in packets), dtype=np.uint8).copy()
    return data, off, ln


def de_bruijn_bytes(length: int) -> bytes:
    """Prefix of the order-2 de Bruijn sequence over 256 symbols: every bigram is
    distinct, so every byte creates the maximum number of model nodes (the
    worst case that first triggers the model reset at 1920 B)."""
    k, n = 256, 2
    a = [0] * (k * n)
    seq = []

    def db(t, p):
        if len(seq) >= length:
            return
        if t > n:
            if n % p == 0:
                seq.extend(a[1 : p + 1])
        else:
            a[t] = a[t - p]
            db(t + 1, p)
            for j in range(a[t - p] + 1, k):
                a[t] = j
                db(t + 1, t)

    db(1, 1)
    return bytes(seq[:length])
