"""Per-step kernel time difference of two rocprofv3 kernel_stats.csv files:
    python tools/prof_diff.py a.csv b.csv steps [name-filter]"""
import csv
import sys

def load(p):
    return {r["Name"]: (float(r["TotalDurationNs"]), int(r["Calls"])) for r in csv.DictReader(open(p))}

a, b = load(sys.argv[1]), load(sys.argv[2])
steps = float(sys.argv[3])
flt = sys.argv[4] if len(sys.argv) > 4 else ""
rows = []
for k in set(a) | set(b):
    if flt and flt not in k:
        continue
    ta, tb = a.get(k, (0, 0))[0], b.get(k, (0, 0))[0]
    rows.append((tb - ta, ta, tb, k))
rows.sort()
print("A total %.2f ms/step  B total %.2f ms/step" % (sum(r[1] for r in rows) / steps / 1e6, sum(r[2] for r in rows) / steps / 1e6))
for d, ta, tb, k in rows[:12] + rows[-12:]:
    print("%+8.3f  %7.3f -> %7.3f ms/step  %s" % (d / steps / 1e6, ta / steps / 1e6, tb / steps / 1e6,
                                               k.replace("void ", "").replace("(anonymous namespace)::", "")[:90]))
