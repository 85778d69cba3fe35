"""Soak run (diagnostic, GPU box): many batches through both entry kinds
against the oracle, counting wrong results and the record-light decoder's
hand-off sum disagreements (enet_rc_debug_counter 7).
usage: python tools/soak.py SECONDS [OUT.json] [PHASE_LOG]
       python tools/soak.py replay SEED N GAME   (one round with those inputs, return codes printed)
SOAK_POOL=k: the rounds draw from k batches made (with their oracle outputs)
at the start instead of a new batch each round -- the same calls, many more
rounds per minute (the oracle's compress on the CPU is most of a round).
PHASE_LOG: the phase about to run is written (and flushed) there before each
step, and every step ends in a device-wide synchronize, so that an
asynchronously reported device error is pinned to the step before it.
Each round: a mixed batch (random packet count 20k-60k, sizes 1-1400 B or
game state), compressed on the device and checked against the oracle by
digest, decompressed from device memory and from host memory (gapped slots:
the GPU gather over the caller's mapped range), each checked byte for byte,
and compressed again from host memory into gapped host slots (checked
against the oracle by digest)."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from enet_amd import RangeCoder, synth  # noqa: E402
from oracle.pyoracle import compress_batch, fnv_digest  # noqa: E402

replay = sys.argv[1] == "replay"
limit = 1e9 if replay else float(sys.argv[1])
out_path = sys.argv[2] if len(sys.argv) > 2 and not replay else None
phase_log = open(sys.argv[3], "w") if len(sys.argv) > 3 and not replay else None
if replay:
    phase_log = sys.stdout


def phase(name):
    if phase_log:
        phase_log.write(f"{time.time() - t0:.1f} {name}\n")
        phase_log.flush()
rc = RangeCoder()
P = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
rng = np.random.default_rng(int(time.time()) & 0xFFFF)
t0 = time.time()
pool = []
for i in range(int(os.environ.get("SOAK_POOL", "0"))):
    sd, nn, gm = int(rng.integers(1, 1 << 30)), int(rng.integers(20000, 60001)), bool(rng.random() < 0.25)
    dd, oo, ll = synth.gamestate_batch(nn, 1200, seed=sd) if gm else synth.mixed_batch(nn, lo=1, hi=1400, seed=sd)
    pool.append((sd, nn, gm, dd, oo, ll, compress_batch(dd, oo, ll, "port")))
if pool:
    print(f"pool of {len(pool)} batches ready", flush=True)
    t0 = time.time()
stats = {"rounds": 0, "packets": 0, "bytes": 0, "compress_mismatch": 0, "device_wrong": 0, "host_wrong": 0,
         "host_compress_mismatch": 0, "host_call_errors": [],
         "sum_disagreements": 0, "lane_handoffs": 0, "seeds": []}
while time.time() - t0 < limit:
    seed = int(rng.integers(1, 1 << 30))
    n = int(rng.integers(20000, 60001))
    game = rng.random() < 0.25
    if replay:
        if stats["rounds"]:
            break
        seed, n, game = int(sys.argv[2]), int(sys.argv[3]), bool(int(sys.argv[4]))
    if pool:
        seed, n, game, d, o, l, (want, wo, wcap, wl) = pool[int(rng.integers(0, len(pool)))]
    phase(f"round {stats['rounds'] + 1} seed {seed} n {n} game {int(game)}: inputs")
    if not pool:
        if game:
            d, o, l = synth.gamestate_batch(n, 1200, seed=seed)
        else:
            d, o, l = synth.mixed_batch(n, lo=1, hi=1400, seed=seed)
        want, wo, wcap, wl = compress_batch(d, o, l, "port")
    phase("h2d")
    din = torch.from_numpy(d).cuda()
    doff = torch.from_numpy(o.astype(np.int64)).cuda()
    dlen = torch.from_numpy(l.astype(np.int32)).cuda()
    cap = (2 * dlen.to(torch.int64) + 64).to(torch.int32)
    coff = torch.zeros(n, dtype=torch.int64, device="cuda")
    coff[1:] = torch.cumsum(cap[:-1].to(torch.int64) + 5, 0)
    cout = torch.zeros(int(coff[-1] + cap[-1]), dtype=torch.uint8, device="cuda")
    clen = torch.zeros(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    phase("device compress")
    rc.compress_batch(din, doff, dlen, cout, coff, cap, clen, max_len=int(l.max()))
    torch.cuda.synchronize()
    cl = clen.cpu().numpy().astype(np.uint32)
    cb, co = cout.cpu().numpy(), coff.cpu().numpy().astype(np.uint64)
    cm = int(not (np.array_equal(cl, wl) and fnv_digest(cb, co, cl) == fnv_digest(want, wo, wl)))
    dout = torch.zeros_like(din)
    dl = torch.zeros(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    phase("device decompress")
    rc.decompress_batch(cout, coff, clen, dout, doff, dlen, dl, max_len=int(cl.max()))
    torch.cuda.synchronize()
    dw = int(not (torch.equal(dl, dlen) and torch.equal(dout, din)))
    stats["sum_disagreements"] += rc.lib.enet_rc_debug_counter(rc.ctx, 7)
    stats["lane_handoffs"] += rc.last_lane_count()
    hout = np.zeros(d.size + 64, np.uint8)
    hl = np.zeros(n, np.uint32)
    l32 = l.astype(np.uint32)
    torch.cuda.synchronize()
    phase("host decompress")
    hrc = rc.lib.enet_rc_decompress_batch_host(rc.ctx, P(cb), P(co), P(cl), n, P(hout), P(o), P(l32), P(hl))
    phase(f"host decompress returned {hrc}, paths {rc.lib.enet_rc_last_host_paths(rc.ctx)} "
          f"split {rc.lib.enet_rc_last_split(rc.ctx)}")
    if hrc != 0:
        stats["host_call_errors"].append([stats["rounds"] + 1, "decompress", hrc, seed, n, int(game)])
    torch.cuda.synchronize()
    stats["sum_disagreements"] += rc.lib.enet_rc_debug_counter(rc.ctx, 7)
    hw = int(not (np.array_equal(hl, l32) and np.array_equal(hout[: d.size], d)))
    torch.cuda.synchronize()
    phase("host compress")
    hco = co.copy()
    hcap = (2 * l32 + 64).astype(np.uint32)
    hcb = np.zeros(int(hco[-1]) + int(hcap[-1]) + 64, np.uint8)
    hcl = np.zeros(n, np.uint32)
    hrc = rc.lib.enet_rc_compress_batch_host(rc.ctx, P(d), P(o), P(l32), n, P(hcb), P(hco), P(hcap), P(hcl))
    phase(f"host compress returned {hrc}, paths {rc.lib.enet_rc_last_host_paths(rc.ctx)}")
    if hrc != 0:
        stats["host_call_errors"].append([stats["rounds"] + 1, "compress", hrc, seed, n, int(game)])
    torch.cuda.synchronize()
    hcm = int(not (np.array_equal(hcl, wl) and fnv_digest(hcb, hco, hcl) == fnv_digest(want, wo, wl)))
    torch.cuda.synchronize()
    phase("checked")
    stats["rounds"] += 1
    stats["packets"] += 4 * n
    stats["bytes"] += 4 * int(l.sum())
    stats["host_compress_mismatch"] += hcm
    stats["compress_mismatch"] += cm
    stats["device_wrong"] += dw
    stats["host_wrong"] += hw
    stats["seeds"].append(seed)
    print(f"round {stats['rounds']} seed {seed} n {n} compress_ok {not cm} device_ok {not dw} host_ok {not hw} "
          f"host_compress_ok {not hcm} "
          f"t {time.time() - t0:.0f}s", flush=True)
stats["seconds"] = round(time.time() - t0, 1)
rc.close()
print(json.dumps({k: v for k, v in stats.items() if k != "seeds"}), flush=True)
if out_path:
    json.dump(stats, open(out_path, "w"), indent=1)
