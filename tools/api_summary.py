"""HIP API calls per profiled training step (rocprofv3 --hip-trace): which ones block the host.
python tools/api_summary.py run_hip_api_trace.csv run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict

api = list(csv.DictReader(open(sys.argv[1])))
ker = list(csv.DictReader(open(sys.argv[2])))
ker.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(ker) if 'adamw' in r['Kernel_Name'].lower()]
bounds = [(int(ker[idx[k]]['Start_Timestamp']), int(ker[idx[k + 1]]['Start_Timestamp']))
          for k in range(len(idx) - 1) if idx[k + 1] - idx[k] > 100][1:]
n = len(bounds)
# host side: the API calls that fall between the first and last profiled AdamW launches' API times
t0, t1 = bounds[0][0], bounds[-1][1]
by, cnt = defaultdict(float), defaultdict(float)
big = []
for r in api:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    if s < t0 - 200_000_000 or s > t1:
        continue
    by[r['Function']] += (e - s) / 1e6 / n
    cnt[r['Function']] += 1 / n
    if e - s > 200_000:
        big.append(((e - s) / 1e3, r['Function']))
print("# HIP API per step over %d steps (host ms, calls)" % n)
for k, v in sorted(by.items(), key=lambda kv: -kv[1])[:25]:
    print("  %8.3f ms  %7.1f  %s" % (v, cnt[k], k))
print("# calls > 200 us:")
agg = defaultdict(lambda: [0, 0.0])
for d, f in big:
    agg[f][0] += 1
    agg[f][1] += d
for f, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print("  %s: %d calls, %.0f us total" % (f, c, d))
