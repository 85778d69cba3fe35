"""Diagnostic: the decompress fixtures through the lane path with each fast
decoder (ENET_RC_DEC=6 / 4, ENET_RC_DEC6_DEBUG) -- prints the mismatches."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["ENET_RC_KERNEL"] = "lane3"
import numpy as np, torch
from tests import golden_io
from tests.test_gpu_parity import _run
from enet_amd import RangeCoder
cases = golden_io.decompress_cases()
sel = [int(x) for x in sys.argv[1:]] or list(range(len(cases)))
with RangeCoder() as rc:
    res = _run(rc, True, [cases[i]["input"] for i in sel], [cases[i]["out_limit"] for i in sel])
bad = [(i, len(cases[i]["input"]), cases[i]["out_limit"], r[0], cases[i]["ret"]) for i, r in zip(sel, res)
       if r[0] != cases[i]["ret"] or (cases[i]["ret"] and r[1] != cases[i]["expect"])]
print(os.environ.get("ENET_RC_DEC"), os.environ.get("ENET_RC_DEC6_DEBUG"), "bad", len(bad), bad[:12])
