"""Idle gaps on the main HIP stream of the profiled training steps (host-launch or cross-stream
waits): python tools/gap_summary.py run_kernel_trace.csv [top]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'adamw' in r['Kernel_Name'].lower()]
steps = [(idx[k], idx[k + 1]) for k in range(len(idx) - 1) if idx[k + 1] - idx[k] > 100][1:]
main = rows[idx[0]]['Stream_Id']


def short(r):
    return r['Kernel_Name'].replace('void ', '').replace('(anonymous namespace)::', '')[:60]


hist = defaultdict(float)
worst = defaultdict(lambda: [0.0, 0])
launches = 0
for a, b in steps:
    ks = [r for r in rows[a:b + 1] if r['Stream_Id'] == main]
    launches += len(ks)
    for p, q in zip(ks, ks[1:]):
        g = (int(q['Start_Timestamp']) - int(p['End_Timestamp'])) / 1e3  # us
        for lim in (5, 20, 100, 1e9):
            if g < lim:
                hist[lim] += g / len(steps) / 1e3
                break
        key = short(p) + '  ->  ' + short(q)
        worst[key][0] += g / len(steps)
        worst[key][1] += 1 / len(steps)
n = len(steps)
print("# main stream %s, %d steps, %.0f launches/step" % (main, n, launches / n))
print("# idle ms/step by gap size: <5us %.2f  5-20us %.2f  20-100us %.2f  >100us %.2f" %
      (hist[5], hist[20], hist[100], hist[1e9]))
for k, (v, c) in sorted(worst.items(), key=lambda kv: -kv[1][0])[:top]:
    print("  %8.1f us  %5.1f x  %s" % (v, c, k))
