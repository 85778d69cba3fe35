"""Diagnostic: PCIe-inclusive round trip (host pointers) of the C2 batch split
over k coder contexts on ONE device (enet_rc_multi_* with the device listed k
times: one host thread and one stream per context, so that one context's
copies overlap another's kernels), pageable and pinned caller buffers."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from enet_amd import get_lib, synth  # noqa: E402

GIB = float(1 << 30)


def main():
    lib = get_lib()
    lib.enet_rc_multi_create.restype = C.c_void_p
    lib.enet_rc_multi_create.argtypes = [C.c_void_p, C.c_size_t]
    lib.enet_rc_multi_destroy.argtypes = [C.c_void_p]
    for f in ("enet_rc_multi_compress_batch_host", "enet_rc_multi_decompress_batch_host"):
        getattr(lib, f).argtypes = [C.c_void_p] + [C.c_void_p] * 3 + [C.c_size_t] + [C.c_void_p] * 4
    d, o, l = synth.random_batch(65536, 1200)
    n = len(l)
    cap = (2 * l.astype(np.int64) + 64).astype(np.uint32)
    coff = np.zeros(n, np.uint64)
    coff[1:] = np.cumsum(cap[:-1], dtype=np.uint64)
    lcap = l.astype(np.uint32)
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    nb = float(l.sum(dtype=np.uint64))
    for kind in ("pageable", "pinned"):
        alloc = (lambda k: np.zeros(k, np.uint8)) if kind == "pageable" else \
            (lambda k: torch.zeros(k, dtype=torch.uint8).pin_memory().numpy())
        src = alloc(d.size)
        src[:] = d
        cout = alloc(int(coff[-1] + cap[-1]))
        dout = alloc(d.size)
        for k in (1, 2, 4):
            devs = (C.c_int * k)(*([0] * k))
            m = lib.enet_rc_multi_create(devs, k)
            clen = np.zeros(n, np.uint32)
            dlen = np.zeros(n, np.uint32)
            best_c = best_d = 1e9
            for _ in range(4):
                t0 = time.perf_counter()
                rc = lib.enet_rc_multi_compress_batch_host(m, p(src), p(o), p(lcap), n, p(cout), p(coff), p(cap), p(clen))
                t1 = time.perf_counter()
                rc |= lib.enet_rc_multi_decompress_batch_host(m, p(cout), p(coff), p(clen), n, p(dout), p(o), p(lcap), p(dlen))
                t2 = time.perf_counter()
                assert rc == 0
                best_c, best_d = min(best_c, t1 - t0), min(best_d, t2 - t1)
            ok = bool(np.array_equal(dlen, lcap) and np.array_equal(dout, d))
            print(f"{kind} contexts={k}: round trip {nb / (best_c + best_d) / GIB:.3f} GiB/s "
                  f"(compress {best_c * 1e3:.2f} ms, decompress {best_d * 1e3:.2f} ms) ok={ok}", flush=True)
            lib.enet_rc_multi_destroy(m)


if __name__ == "__main__":
    main()
