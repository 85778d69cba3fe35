#!/usr/bin/env python3
"""Generates tests/golden/* from the REAL reference compress.c.

Run in the build container (where /root/reference exists):

    make -C oracle            # builds oracle/_ref/libenet_ref.so from the reference sources
    python tests/golden/make_golden.py

Every expected value below is produced by calling the reference's own
enet_range_coder_compress / enet_range_coder_decompress (compress.c:246-627)
through ctypes.  The outputs are data fixtures only (inputs + expected
outputs); no reference source is stored.  The reference has no tests or
fixtures of its own, so these vectors are the parity pin.

Files:
  compress_cases.npz    single-buffer compress: input, in_limit, out_limit -> ret, bytes
  gather_cases.npz      multi-buffer compress (incl. empty buffers)        -> ret, bytes
  decompress_cases.npz  decompress of valid / truncated / bit-flipped / garbage streams
  digests.json          C1 / C2 / C3 batch digests (SURVEY.md §8c format)
  crc_cases.npz         enet_crc32 (packet.c:143-163) of single buffers, from the
                        reference library's exported enet_crc32

`python tests/golden/make_golden.py crc` regenerates crc_cases.npz only.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from enet_amd import synth  # noqa: E402
from oracle.pyoracle import Coder, compress_batch, crc32_batch, fnv_digest, have_reference  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def _pack_cases(cases, fields):
    """cases: list of dicts with bytes fields 'input'/'expect' and int fields."""
    blob_in = b"".join(c["input"] for c in cases)
    blob_out = b"".join(c["expect"] for c in cases)
    in_len = np.array([len(c["input"]) for c in cases], dtype=np.uint32)
    ex_len = np.array([len(c["expect"]) for c in cases], dtype=np.uint32)
    arrs = dict(
        inputs=np.frombuffer(blob_in, dtype=np.uint8),
        in_len=in_len,
        expects=np.frombuffer(blob_out, dtype=np.uint8),
        ex_len=ex_len,
    )
    for f in fields:
        arrs[f] = np.array([c[f] for c in cases], dtype=np.int64)
    return arrs


def make_crc():
    """CRC-32 fixtures: every length 0..80, then assorted sizes to 4096 B, plus
    the standard check string; expected values from the reference itself."""
    inputs = [b"123456789", b"", b"\0" * 1200, b"\xff" * 4096]
    for n in range(0, 81):
        inputs.append(synth.random_bytes(n, 500 + n).tobytes())
    for k, n in enumerate((127, 128, 129, 255, 256, 1000, 1023, 1024, 1025, 1199, 1200, 1392,
                           2047, 2048, 2049, 3000, 4095, 4096)):
        inputs.append(synth.random_bytes(n, 900 + k).tobytes())
    blob = np.frombuffer(b"".join(inputs), dtype=np.uint8)
    ln = np.array([len(x) for x in inputs], dtype=np.uint32)
    off = np.concatenate([[0], np.cumsum(ln[:-1], dtype=np.uint64)]).astype(np.uint64)
    crc = crc32_batch(blob, off, ln, kind="reference")
    np.savez_compressed(os.path.join(OUT, "crc_cases.npz"), inputs=blob, in_len=ln,
                        crc=crc.astype(np.int64))
    print(f"crc {len(inputs)}  check('123456789') = {int(crc[0]):#010x}")


def main():
    if not have_reference():
        sys.exit("oracle/_ref/libenet_ref.so missing: run `make -C oracle` first")
    if sys.argv[1:] == ["crc"]:
        make_crc()
        return
    make_crc()
    if not have_reference():
        sys.exit("oracle/_ref/libenet_ref.so missing: run `make -C oracle` first")
    ref = Coder("reference")
    rng_seed = 0x1234

    # ------------------------------------------------------------- compress
    inputs = []
    kats = [b"\x5a", b"hello world", b"\0" * 1200,
            bytes(((i * 37) ^ 0x5A) & 0xFF for i in range(64)), bytes(range(256))]
    inputs += kats
    sizes = [1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 31, 63, 64, 65, 100, 127, 128, 255, 256, 257,
             500, 777, 1000, 1199, 1200, 1201, 1392, 1500, 2048, 3000, 4000, 4095, 4096]
    for k, n in enumerate(sizes):
        inputs.append(synth.random_bytes(n, rng_seed + k).tobytes())
    gd, go, gl = synth.gamestate_batch(8, 1200)
    inputs += [gd[int(go[i]): int(go[i]) + int(gl[i])].tobytes() for i in range(8)]
    gd, go, gl = synth.gamestate_batch(4, 4096, seed=77)
    inputs += [gd[int(go[i]): int(go[i]) + int(gl[i])].tobytes() for i in range(4)]
    # model reset boundary (first reset at 1920 B of de Bruijn input)
    inputs += [synth.de_bruijn_bytes(n) for n in (1000, 1919, 1920, 1921, 2500, 4096)]
    # rescale-heavy and degenerate inputs
    inputs += [b"\0" * 4096, b"\xff" * 3000, bytes([7]) * 255, b"ab" * 2000,
               bytes(i & 0xFF for i in range(4096)), bytes((i * i) & 0xFF for i in range(4096)),
               bytes((255 - i) & 0xFF for i in range(256)) * 8,
               bytes([0, 1]) * 700 + bytes(range(256)) * 4]
    # small-alphabet random data (long contexts, many rescales)
    for k, alpha in enumerate((2, 3, 4, 16)):
        r = synth.random_bytes(3000, 99 + k)
        inputs.append((r % alpha).astype(np.uint8).tobytes())

    ccases = []
    for data in inputs:
        n = len(data)
        for out_limit in sorted({2 * n + 64, n}):
            ret, out = ref.compress(data, out_limit=out_limit)
            ccases.append(dict(input=data, expect=out, ret=ret, in_limit=n, out_limit=out_limit))
        # a tight limit: exactly the needed size, and one less
        ret, out = ref.compress(data, out_limit=2 * n + 64)
        for lim in (ret, ret - 1):
            if lim >= 0:
                r2, o2 = ref.compress(data, out_limit=lim)
                ccases.append(dict(input=data, expect=o2, ret=r2, in_limit=n, out_limit=lim))
    # in_limit is only checked for > 0 (compress.c:257)
    d = inputs[8]
    for il in (0, 1, 5):
        r2, o2 = ref.compress(d, in_limit=il)
        ccases.append(dict(input=d, expect=o2, ret=r2, in_limit=il, out_limit=2 * len(d) + 64))
    # empty input
    r2, o2 = ref.compress(b"", in_limit=0)
    ccases.append(dict(input=b"", expect=o2, ret=r2, in_limit=0, out_limit=64))
    np.savez_compressed(os.path.join(OUT, "compress_cases.npz"),
                        **_pack_cases(ccases, ["ret", "in_limit", "out_limit"]))

    # --------------------------------------------------------------- gather
    gcases = []
    base = synth.random_bytes(1400, 4242).tobytes()
    splits = [
        [(0, 1200)],
        [(0, 600), (600, 600)],
        [(0, 4), (4, 44), (48, 1000), (1048, 152)],
        [(0, 0), (0, 64)],                       # empty first buffer: skipped
        [(0, 32), (32, 0), (32, 32)],            # empty middle buffer: phantom byte
        [(0, 32), (32, 32), (64, 0)],            # empty last buffer: phantom byte
        [(0, 0), (0, 0), (5, 10)],               # empty first and second
        [(i * 20, 20) for i in range(64)],       # ENET_BUFFER_MAXIMUM-1 = 64 entries
        [(0, 1), (1, 1), (2, 1), (3, 1)],
    ]
    for spans in splits:
        tot = sum(l for _, l in spans)
        for out_limit in (2 * tot + 70, tot):
            ret, out = ref.compress_gather(base, spans, max(tot, 1), out_limit)
            gcases.append(dict(input=b"", expect=out, ret=ret, out_limit=out_limit,
                               in_limit=max(tot, 1), spans=spans))
    garr = _pack_cases(gcases, ["ret", "out_limit", "in_limit"])
    span_flat, span_cnt = [], []
    for c in gcases:
        span_cnt.append(len(c["spans"]))
        span_flat += [v for s in c["spans"] for v in s]
    garr["backing"] = np.frombuffer(base, dtype=np.uint8)
    garr["spans"] = np.array(span_flat, dtype=np.int64)
    garr["span_cnt"] = np.array(span_cnt, dtype=np.int64)
    np.savez_compressed(os.path.join(OUT, "gather_cases.npz"), **garr)

    # ----------------------------------------------------------- decompress
    dcases = []
    valid = [c for c in ccases if c["ret"] > 0 and c["out_limit"] == 2 * len(c["input"]) + 64]
    for c in valid:
        n = len(c["input"])
        for out_limit in sorted({4096, n, max(n - 1, 0)}):
            ret, out = ref.decompress(c["expect"], out_limit)
            dcases.append(dict(input=c["expect"], expect=out, ret=ret, out_limit=out_limit))
    # corrupt streams: truncation, bit flips, garbage
    frng = np.random.default_rng(20251015)
    streams = [c["expect"] for c in valid]
    for t in range(1500):
        s = bytearray(streams[t % len(streams)])
        kind = t % 3
        if kind == 0 and len(s) > 1:
            s = s[: frng.integers(1, len(s))]
        elif kind == 1:
            for _ in range(int(frng.integers(1, 4))):
                pos = int(frng.integers(0, len(s)))
                s[pos] ^= 1 << int(frng.integers(0, 8))
        else:
            s = bytearray(frng.integers(0, 256, size=int(frng.integers(1, 300)), dtype=np.uint8).tobytes())
        for out_limit in (4096, 300):
            ret, out = ref.decompress(bytes(s), out_limit)
            dcases.append(dict(input=bytes(s), expect=out, ret=ret, out_limit=out_limit))
    # empty / tiny inputs
    for s in (b"", b"\0", b"\xff", b"\0\0\0\0", b"\xff\xff\xff\xff", b"\x01\x02\x03"):
        ret, out = ref.decompress(s, 4096)
        dcases.append(dict(input=s, expect=out, ret=ret, out_limit=4096))
    np.savez_compressed(os.path.join(OUT, "decompress_cases.npz"),
                        **_pack_cases(dcases, ["ret", "out_limit"]))

    # -------------------------------------------------------------- digests
    digests = {}
    for name, (d, o, l) in {
        "C1_random_4096x256": synth.random_batch(4096, 256),
        "C2_random_65536x1200": synth.random_batch(65536, 1200),
        "C3_gamestate_65536x1200": synth.gamestate_batch(65536, 1200),
    }.items():
        out, oo, cap, ol = compress_batch(d, o, l, kind="reference")
        digests[name] = dict(packets=int(len(l)), in_bytes=int(l.sum(dtype=np.uint64)),
                             out_bytes=int(ol.sum(dtype=np.uint64)),
                             input_fnv=fnv_digest(d, o, l),
                             digest=fnv_digest(out, oo, ol),
                             out_limit="2N+64")
        print(name, digests[name], flush=True)
    with open(os.path.join(OUT, "digests.json"), "w") as f:
        json.dump(digests, f, indent=2)
    print(f"compress {len(ccases)}  gather {len(gcases)}  decompress {len(dcases)}")


if __name__ == "__main__":
    main()
