"""In-process interleaved A/B timing of several builds of the library.

usage: python tools/abx.py A B [C ...] [--workload c2] [--rounds 12]
Loads enet_amd/lib/libenet_rc_amd_<X>.so for every X (RTLD_LOCAL, one
context each), then alternates compress + decompress launches of the builds
round by round on the same device-resident batch, timing each launch with HIP
events.  Clock drift on the box hits every build alike, so medians of the
per-round ratios are much tighter than separate bench.py processes.
Prints one JSON line: per build the median compress/decompress ms and GiB/s,
and the round-trip ratio to the first build.
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load(tag):
    lib = C.CDLL(os.path.join(ROOT, "enet_amd", "lib", f"libenet_rc_amd_{tag}.so"), mode=C.RTLD_LOCAL)
    vp, sz, u32 = C.c_void_p, C.c_size_t, C.c_uint32
    lib.enet_range_coder_create.restype = vp
    for f in (lib.enet_rc_compress_batch_device, lib.enet_rc_decompress_batch_device):
        f.restype = C.c_int
        f.argtypes = [vp, vp, vp, vp, sz, u32, vp, vp, vp, vp, vp]
    return lib, lib.enet_range_coder_create()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tags", nargs="+")
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--rounds", type=int, default=12)
    a = ap.parse_args()
    import torch
    from enet_amd import synth
    gen = {"c2": synth.random_batch, "c3": synth.gamestate_batch}[a.workload]
    d, o, l = gen(65536, 1200)
    dev = torch.device("cuda", 0)
    din = torch.from_numpy(d).to(dev)
    doff = torch.from_numpy(o.astype(np.int64)).to(dev)
    dlen = torch.from_numpy(l.astype(np.int32)).to(dev)
    n = len(l)
    cap = (2 * dlen.to(torch.int64) + 64).to(torch.int32)
    coff = torch.zeros(n, dtype=torch.int64, device=dev)
    coff[1:] = torch.cumsum(cap[:-1].to(torch.int64), 0)
    cout = torch.empty(int(coff[-1] + cap[-1]), dtype=torch.uint8, device=dev)
    clen = torch.zeros(n, dtype=torch.int32, device=dev)
    dout = torch.empty_like(din)
    dl = torch.zeros(n, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)
    sp = C.c_void_p(st.cuda_stream)
    libs = {}
    for t in a.tags:                       # "X@k": a k-th context of build X (same code object)
        base = t.split("@")[0]
        lib = libs[base][0] if base in libs else load(base)[0]
        libs[t] = (lib, lib.enet_range_coder_create())
    in_bytes = int(l.sum(dtype=np.uint64))

    def run(t, ev):
        lib, ctx = libs[t]
        ev[0].record(st)
        rc = lib.enet_rc_compress_batch_device(ctx, din.data_ptr(), doff.data_ptr(), dlen.data_ptr(), n, 1200,
                                               cout.data_ptr(), coff.data_ptr(), cap.data_ptr(), clen.data_ptr(), sp)
        ev[1].record(st)
        rc |= lib.enet_rc_decompress_batch_device(ctx, cout.data_ptr(), coff.data_ptr(), clen.data_ptr(), n, 2464,
                                                  dout.data_ptr(), doff.data_ptr(), dlen.data_ptr(), dl.data_ptr(), sp)
        ev[2].record(st)
        assert rc == 0

    ok = {}
    for t in a.tags:                                   # warm-up + correctness per build
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        run(t, ev)
        run(t, ev)
        torch.cuda.synchronize()
        ok[t] = bool(torch.equal(dl, dlen)) and bool(torch.equal(dout, din))
        dout.zero_()
    res = {t: ([], []) for t in a.tags}
    for r in range(a.rounds):
        order = a.tags if r % 2 == 0 else a.tags[::-1]
        evs = {t: [torch.cuda.Event(enable_timing=True) for _ in range(3)] for t in order}
        for t in order:
            run(t, evs[t])
        torch.cuda.synchronize()
        for t in order:
            e = evs[t]
            res[t][0].append(e[0].elapsed_time(e[1]))
            res[t][1].append(e[1].elapsed_time(e[2]))
    base = a.tags[0]
    out = {"workload": a.workload, "rounds": a.rounds}
    for t in a.tags:
        c, dd = res[t]
        rt = [x + y for x, y in zip(c, dd)]
        brt = [x + y for x, y in zip(*res[base])]
        out[t] = {"ok": ok[t], "comp_ms": round(statistics.median(c), 4), "dec_ms": round(statistics.median(dd), 4),
                  "rt_GiBps": round(in_bytes / (statistics.median(rt) / 1e3) / 2**30, 4),
                  "rt_ratio_vs_" + base: round(statistics.median([b / x for b, x in zip(brt, rt)]), 4),
                  "comp_ratio": round(statistics.median([b / x for b, x in zip(res[base][0], c)]), 4),
                  "dec_ratio": round(statistics.median([b / x for b, x in zip(res[base][1], dd)]), 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
