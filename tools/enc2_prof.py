"""Per-phase cycles of the two-pass encoder's scan pass (diagnostic build,
make -C enet_amd/csrc e2prof).  Runs one C2 compress batch and prints the
shader cycles each phase took, summed over wavefronts, per packet."""
import ctypes as C
import os
import sys

os.environ["ENET_RC_LIB"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "enet_amd", "lib",
                                         os.environ.get("E2_LIB", "libenet_rc_amd_e2prof.so"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from enet_amd import RangeCoder, compress_batch, synth, get_lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
lib = get_lib()
lib.rc_enc2_prof_read.restype = C.c_int
lib.rc_enc2_prof_read.argtypes = [C.c_void_p, C.c_int]
d, o, l = (synth.gamestate_batch if len(sys.argv) > 2 and sys.argv[2] == "c3" else synth.random_batch)(n, 1200)
din = torch.from_numpy(d).cuda()
doff = torch.from_numpy(o.astype("int64")).cuda()
dlen = torch.from_numpy(l.astype("int32")).cuda()
buf = (C.c_ulonglong * 32)()
with RangeCoder() as rc:
    compress_batch(rc, din, doff, dlen, max_len=1200)
    torch.cuda.synchronize()
    lib.rc_enc2_prof_read(buf, 1)
    compress_batch(rc, din, doff, dlen, max_len=1200)
    torch.cuda.synchronize()
    lib.rc_enc2_prof_read(buf, 1)
names = ["load+zero", "hist+bigrams", "sizes", "scatter", "exceptional", "plain+end", "prefetch", "-"]
tot = sum(buf[k] for k in range(8))
for k, nm in enumerate(names):
    print(f"{nm:14s} {buf[k] / n:10.0f} cycles/packet  {100.0 * buf[k] / max(tot, 1):5.1f} %")
print(f"{'total':14s} {tot / n:10.0f} cycles/packet")
# the code pass: cycles per wavefront-step (one position of each of the wave's 64 packets)
cnames = ["loop/loads", "record+root lookup", "code 1 (sub)", "code 2 (o1 after o2)", "root add+update",
          "code 3 (root)", "rescale chk+ring", "-"]
steps = (n // 64) * 1200
ctot = sum(buf[8 + k] for k in range(8))
for k, nm in enumerate(cnames):
    print(f"code {nm:22s} {buf[8 + k] / steps:8.0f} cycles/wave-step  {100.0 * buf[8 + k] / max(ctot, 1):5.1f} %")
print(f"code {'total':22s} {ctot / steps:8.0f} cycles/wave-step")
# the two-wavefront code pass (rc_enc2_code2): per wavefront and part of 4 positions
parts = (n // 64) * 1200 / 4
print(f"code2 helper work {buf[8] / parts:7.0f}  barrier wait {buf[9] / parts:7.0f} cycles/wave-part")
print(f"code2 coder  work {buf[10] / parts:7.0f}  barrier wait {buf[11] / parts:7.0f} cycles/wave-part")

# the wide scan (rc_enc2_wscan): cycles per packet it took
wnames = ["load+zero", "bucket sizes", "starts+pad", "scatter", "small buckets", "big: sort",
          "big: short runs", "big: dense o2", "big: o1 list", "big: dense o1", "end", "-"]
wtot = sum(buf[16 + k] for k in range(12))
if wtot:
    for k, nm in enumerate(wnames):
        print(f"wide {nm:16s} {buf[16 + k] / n:10.0f} cycles/packet  {100.0 * buf[16 + k] / wtot:5.1f} %")
    print(f"wide {'total':16s} {wtot / n:10.0f} cycles/packet")
