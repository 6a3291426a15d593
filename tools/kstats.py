"""Average duration per kernel of a rocprofv3 --stats kernel_stats.csv, filtered by a name part:
    python tools/kstats.py STATS_CSV NAME_PART [label]"""
import csv
import re
import sys

path, part = sys.argv[1], sys.argv[2]
label = sys.argv[3] if len(sys.argv) > 3 else ""
for r in csv.DictReader(open(path)):
    if part in r["Name"]:
        n = re.sub(r"\(anonymous namespace\)::", "", r["Name"])
        n = re.split(r"\((?!anon)", n)[0].replace("void ", "")[:110]
        print(f"{label:>6} {float(r['AverageNs']) / 1e3:9.1f} us x{int(r['Calls']):3d}  {n}")
