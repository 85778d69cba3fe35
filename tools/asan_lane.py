"""Diagnostic (host only): a batch through the lane kernels' per-lane logic
under AddressSanitizer (tools/asan/lane_asan.cpp), each packet in buffers of
exactly its size.  usage: python tools/asan_lane.py KIND SEED N [v3|v6|v6s ...]
KIND: mixed (sizes 1-1400) or game (game state, 1200 B)."""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from enet_amd import synth  # noqa: E402
from oracle.pyoracle import compress_batch  # noqa: E402

kind, seed, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
variants = sys.argv[4:] or ["v3", "v6s"]
d, o, l = synth.gamestate_batch(n, 1200, seed=seed) if kind == "game" else synth.mixed_batch(n, lo=1, hi=1400, seed=seed)
want, wo, wcap, wl = compress_batch(d, o, l, "port")
tmp = tempfile.mkdtemp(prefix="lane_asan_")
d.tofile(os.path.join(tmp, "data.bin"))
l.astype(np.uint32).tofile(os.path.join(tmp, "dlen.bin"))
np.concatenate([want[int(wo[i]): int(wo[i]) + int(wl[i])] for i in range(n)]).tofile(os.path.join(tmp, "comp.bin"))
wl.astype(np.uint32).tofile(os.path.join(tmp, "clen.bin"))
# alignment phases as in tools/soak.py: the payload back to back, compressed slots 2 len + 64 + 5 apart
coff = np.zeros(n, np.int64)
coff[1:] = np.cumsum(2 * l[:-1].astype(np.int64) + 64 + 5)
np.stack([o.astype(np.int64) & 15, coff & 15], axis=1).astype(np.uint8).tofile(os.path.join(tmp, "phases.bin"))
flags = {"v3": [], "v6": ["-DDEC6"], "v6s": ["-DDEC6", "-DDEC6S"]}
csrc = os.path.join(ROOT, "enet_amd", "csrc")
rc = 0
for v in variants:
    exe = os.path.join(tmp, "lane_asan_" + v)
    subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer"] +
                          flags[v] + ["-I", csrc, "-I", os.path.join(ROOT, "tests", "proto"), "-o", exe,
                                      os.path.join(ROOT, "tools", "asan", "lane_asan.cpp")])
    r = subprocess.run([exe, tmp], capture_output=True, text=True)
    print(v, kind, seed, n, r.returncode, r.stdout.strip(), r.stderr[-3000:])
    rc |= r.returncode
sys.exit(rc)
