"""Timeline of the last bursts of GPU work in a rocprofv3 trace directory
(kernel_trace + memory_copy_trace CSVs): bursts are separated by >= GAP ms
with nothing running; each event with start / end (ms from the burst's
start), queue, thread, name.  usage: python tools/timeline.py DIR [bursts] [gap_ms]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 2
gap = float(sys.argv[3]) if len(sys.argv) > 3 else 0.5
ev = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "q%s" % r["Queue_Id"],
                   "t%s" % r["Thread_Id"][-3:], r["Kernel_Name"].split("(")[0][:48]))
for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "s%s" % r["Stream_Id"], "dma",
                   r["Direction"].replace("MEMORY_COPY_", "")))
ev.sort()
bursts, cur, end = [], [], 0
for e in ev:
    if cur and e[0] - end > gap * 1e6:
        bursts.append(cur)
        cur = []
    cur.append(e)
    end = max(end, e[1]) if len(cur) > 1 else e[1]
if cur:
    bursts.append(cur)
if os.environ.get("TL_SUMMARY"):
    for i, b in enumerate(bursts):
        t0 = b[0][0]
        print(f"burst {i}: {len(b)} events, {(max(e[1] for e in b) - t0) / 1e6:.3f} ms")
    sel = [int(x) for x in os.environ["TL_SUMMARY"].split(",") if x]
    bursts = [bursts[i] for i in sel]
    nb = len(bursts)
for b in bursts[-nb:]:
    t0 = b[0][0]
    t1 = max(e[1] for e in b)
    print(f"--- burst {len(b)} events, {(t1 - t0) / 1e6:.3f} ms")
    for s, e, q, th, name in b:
        print(f"{(s - t0) / 1e6:8.3f} {(e - t0) / 1e6:8.3f} {(e - s) / 1e6:7.3f} {q:>4} {th:>5} {name}")
