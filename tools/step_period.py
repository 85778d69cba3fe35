"""Per-step period of bench.py's round trips from a rocprofv3 kernel trace:
the interval between consecutive starts of a marker kernel (default
rc_decompress_dec6s), median and min over the trace, in microseconds.
usage: python tools/step_period.py run_kernel_trace.csv [kernel]"""
import csv
import statistics
import sys

k = sys.argv[2] if len(sys.argv) > 2 else "rc_decompress_dec6s"
st = sorted(int(r["Start_Timestamp"]) for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"].startswith(k))
d = [(b - a) / 1e3 for a, b in zip(st, st[1:])]
# (the warm-up and the bench's own correctness checks sit between some starts: the shortest half)
d = sorted(d)[: max(1, len(d) // 2 + 1)]
print(f"{k}: {len(st)} starts, step period median {statistics.median(d):.1f} us, min {min(d):.1f} us")
