"""Readers for the committed golden fixtures (tests/golden/*.npz, made by make_golden.py)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _unpack(path, fields):
    z = np.load(path, allow_pickle=False)
    ins, inl = z["inputs"], z["in_len"]
    exs, exl = z["expects"], z["ex_len"]
    io = np.concatenate([[0], np.cumsum(inl.astype(np.int64))])
    eo = np.concatenate([[0], np.cumsum(exl.astype(np.int64))])
    cases = []
    for i in range(len(inl)):
        c = dict(input=ins[io[i]:io[i + 1]].tobytes(), expect=exs[eo[i]:eo[i + 1]].tobytes())
        for f in fields:
            c[f] = int(z[f][i])
        cases.append(c)
    return cases, z


def compress_cases():
    return _unpack(os.path.join(GOLDEN, "compress_cases.npz"), ["ret", "in_limit", "out_limit"])[0]


def decompress_cases():
    return _unpack(os.path.join(GOLDEN, "decompress_cases.npz"), ["ret", "out_limit"])[0]


def gather_cases():
    cases, z = _unpack(os.path.join(GOLDEN, "gather_cases.npz"), ["ret", "out_limit", "in_limit"])
    backing = z["backing"].tobytes()
    spans, cnt = z["spans"], z["span_cnt"]
    k = 0
    for c, n in zip(cases, cnt):
        c["spans"] = [(int(spans[k + 2 * j]), int(spans[k + 2 * j + 1])) for j in range(int(n))]
        k += 2 * int(n)
        c["backing"] = backing
    return cases


def digests():
    with open(os.path.join(GOLDEN, "digests.json")) as f:
        return json.load(f)


def crc_cases():
    """[(input bytes, expected enet_crc32 value)] from crc_cases.npz."""
    z = np.load(os.path.join(GOLDEN, "crc_cases.npz"), allow_pickle=False)
    ins, inl, crc = z["inputs"], z["in_len"], z["crc"]
    io = np.concatenate([[0], np.cumsum(inl.astype(np.int64))])
    return [(ins[io[i]:io[i + 1]].tobytes(), int(crc[i])) for i in range(len(inl))]
