"""Per-stream kernel time of the profiled training steps: python tools/stream_summary.py run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'adamw' in r['Kernel_Name'].lower()]
steps = [(idx[k], idx[k + 1]) for k in range(len(idx) - 1) if idx[k + 1] - idx[k] > 100][1:]
print("# per-step kernel time by HIP stream (0 = main, 1 = side: weight gradients, parameter-gradient")
print("# tails, discarded branches), averaged over %d profiled steps; span = AdamW-to-AdamW wall time" % len(steps))
span = sum((int(rows[b]['End_Timestamp']) - int(rows[a]['End_Timestamp'])) / 1e6 for a, b in steps) / len(steps)
print("span_ms %.2f" % span)
for sid in sorted({r['Stream_Id'] for r in rows}):
    by, n = defaultdict(float), defaultdict(float)
    for a, b in steps:
        for r in rows[a + 1:b + 1]:
            if r['Stream_Id'] != sid:
                continue
            k = r['Kernel_Name'].replace('void ', '').replace('(anonymous namespace)::', '')[:90]
            by[k] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 / len(steps)
            n[k] += 1 / len(steps)
    print("stream %s busy_ms %.2f" % (sid, sum(by.values())))
    for k, v in sorted(by.items(), key=lambda kv: -kv[1])[:25]:
        print("  %7.3f ms  %5.1f calls  %s" % (v, n[k], k))
