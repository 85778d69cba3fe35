"""CRC-32 kernel timing on C2 and C4 batches (bench.py's crc32 leg on its own).
usage: python tools/crc_time.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402
from enet_amd import RangeCoder, synth  # noqa: E402

coder = RangeCoder()
stream = torch.cuda.current_stream()
for name, (d, o, l) in {"c2": synth.random_batch(65536, 1200), "c4": synth.mixed_batch(1 << 20)}.items():
    din = torch.from_numpy(d).cuda()
    doff = torch.from_numpy(o.astype("int64")).cuda()
    dlen = torch.from_numpy(l.astype("int32")).cuda()
    r = bench.crc32_bench(coder, din, doff, dlen, int(l.sum()), len(l), stream)
    print(json.dumps({"workload": name, **r}))
coder.close()
