"""Batch latency vs batch size, device-resident, 1200-B packets: lane kernels
for every size (ENET_RC_SMALL_BATCH=0) vs the default routing (batches that fit
on the chip at one wavefront per packet go to the wave kernel, rc_kernels.hip
launch()).  Decompress passes max_len=0 (inputs of random packets exceed 1200 B);
"bounded" is the default routing with the output bound (max_out=1200,
enet_rc_decompress_batch_device_bounded) that sizes the wave decoder's model."""
import json, os, sys, time
sys.path.insert(0, ".")
import numpy as np
import torch
from enet_amd import RangeCoder, synth

def coder(kind):
    if kind == "lanes":
        os.environ["ENET_RC_SMALL_BATCH"] = "0"
    c = RangeCoder()
    os.environ.pop("ENET_RC_SMALL_BATCH", None)
    return c

dev = torch.device("cuda:0")
coders = {k: coder(k) for k in ("lanes", "auto")}
coders["bounded"] = coders["auto"]
for gen in ("random", "game"):
    for n in [int(x) for x in os.environ.get("SB_SIZES", "1,64,256,512,1024,1280,2048").split(",")]:
        d, o, l = (synth.random_batch if gen == "random" else synth.gamestate_batch)(n, 1200)
        din = torch.from_numpy(np.ascontiguousarray(d)).to(dev)
        doff = torch.from_numpy(o.astype(np.int64)).to(dev)
        dlen = torch.from_numpy(l.astype(np.int32)).to(dev)
        cap = 2 * 1200 + 64
        oo = torch.arange(n, dtype=torch.int64, device=dev) * cap
        ocap = torch.full((n,), cap, dtype=torch.int32, device=dev)
        out = torch.empty(n * cap, dtype=torch.uint8, device=dev)
        olen = torch.empty(n, dtype=torch.int32, device=dev)
        back = torch.empty(n * 1200, dtype=torch.uint8, device=dev)
        blen = torch.empty(n, dtype=torch.int32, device=dev)
        bcap = torch.full((n,), 1200, dtype=torch.int32, device=dev)
        row = {"gen": gen, "n": n}
        ref = None
        for k, c in coders.items():
            best_c = best_d = 1e9
            for rep in range(3):
                torch.cuda.synchronize(); t0 = time.perf_counter()
                c.compress_batch(din, doff, dlen, out, oo, ocap, olen, max_len=1200)
                torch.cuda.synchronize(); t1 = time.perf_counter()
                c.decompress_batch(out, oo, olen, back, doff, bcap, blen, max_len=0,
                                   max_out=1200 if k == "bounded" else 0)
                torch.cuda.synchronize(); t2 = time.perf_counter()
                best_c, best_d = min(best_c, t1 - t0), min(best_d, t2 - t1)
            ok = bool(torch.equal(back, din)) and bool((blen == 1200).all())
            sig = olen.cpu().numpy().tobytes()
            ref = ref or sig
            row[k] = {"compress_ms": round(best_c * 1e3, 3), "decompress_ms": round(best_d * 1e3, 3),
                      "ok": ok and sig == ref}
        print(json.dumps(row), flush=True)
