import sys, json
sys.path.insert(0, ".")
import bench
from enet_amd import RangeCoder, synth
d, o, l = synth.random_batch(256, 1200)
c = RangeCoder()
print(json.dumps(bench.per_datagram_call(c, d, o, l)))
gd, go, gl = synth.gamestate_batch(256, 1200)
print(json.dumps(bench.per_datagram_call(c, gd, go, gl)))
