"""The helper wavefronts' passes in rc_decompress_dec6s on C2 (a
-DDEC6_HELP_COUNT build, ENET_RC_LIB=.../libenet_rc_amd_hcount.so): busy and
idle passes per launch (ws.counters[5..6]), for splitting the kernel's PMC
instruction counts between helper and decoding wavefronts with the static
per-pass costs of tools/dec6_helper_cost.py."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from enet_amd import RangeCoder, synth  # noqa: E402

d, o, l = synth.random_batch(65536, 1200)
rc = RangeCoder()
din = torch.from_numpy(d).cuda()
doff = torch.from_numpy(o.astype(np.int64)).cuda()
dlen = torch.from_numpy(l.astype(np.int32)).cuda()
n = len(l)
cap = (2 * dlen.to(torch.int64) + 64).to(torch.int32)
coff = torch.zeros(n, dtype=torch.int64, device="cuda")
coff[1:] = torch.cumsum(cap[:-1].to(torch.int64), 0)
cout = torch.empty(int(coff[-1] + cap[-1]), dtype=torch.uint8, device="cuda")
clen = torch.zeros(n, dtype=torch.int32, device="cuda")
rc.compress_batch(din, doff, dlen, cout, coff, cap, clen, max_len=1200)
dout = torch.empty_like(din)
dl = torch.zeros(n, dtype=torch.int32, device="cuda")
res = []
for _ in range(3):
    rc.decompress_batch(cout, coff, clen, dout, doff, dlen, dl, max_len=int(clen.max().item()))
    torch.cuda.synchronize()
    res.append((rc.lib.enet_rc_debug_counter(rc.ctx, 5), rc.lib.enet_rc_debug_counter(rc.ctx, 6)))
ok = bool(torch.equal(dout, din))
print(json.dumps({"helper_busy_passes": [r[0] for r in res], "helper_idle_passes": [r[1] for r in res],
                  "helper_waves": 1024, "decoding_waves": 1024, "roundtrip_ok": ok}))
