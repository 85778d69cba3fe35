"""Interleaved A/B of environment settings on bench.py's PCIe-inclusive leg
(host-pointer batches), one process per run.
usage: python tools/pcie_ab.py ROUNDS "ENV=A ..." "ENV=B ..." ...  -> one line per run"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r"""
import json, sys
sys.path.insert(0, %r)
import bench
from enet_amd import RangeCoder, synth
class A: pass
c = RangeCoder()
d, o, l = synth.random_batch(65536, 1200)
r = bench.pcie_inclusive(c, d, o, l, A())
print(json.dumps({k: r[k] for k in ("value", "compress_GiBps", "decompress_GiBps", "bit_exact")}))
""" % ROOT

rounds = int(sys.argv[1])
for r in range(rounds):
    for spec in sys.argv[2:]:
        env = dict(os.environ)
        for kv in spec.split():
            k, v = kv.split("=", 1)
            env[k] = v
        out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=300)
        line = [x for x in out.stdout.splitlines() if x.startswith("{")]
        print(r, spec, line[-1] if line else out.stderr[-500:], flush=True)
