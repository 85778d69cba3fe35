"""Per-datagram call latency vs datagram size (fixed overhead + per-byte slope)."""
import sys, json
sys.path.insert(0, ".")
import bench
from enet_amd import RangeCoder, synth
c = RangeCoder()
for n in (1, 16, 150, 600, 1200):
    d, o, l = synth.random_batch(256, n)
    r = bench.per_datagram_call(c, d, o, l)
    print(json.dumps(r), flush=True)
