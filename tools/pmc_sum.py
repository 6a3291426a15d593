"""Summarise rocprofv3 --pmc counter_collection.csv files: mean counter value per dispatch
of kernels whose name contains a filter.   python tools/pmc_sum.py filter file.csv [...]"""
import csv
import sys
from collections import defaultdict

flt = sys.argv[1]
tot = defaultdict(float)
disp = defaultdict(set)
for path in sys.argv[2:]:
    for row in csv.DictReader(open(path)):
        if flt not in row["Kernel_Name"]:
            continue
        c = row["Counter_Name"]
        tot[c] += float(row["Counter_Value"])
        disp[c].add(row["Dispatch_Id"])
for c in sorted(tot):
    print(f"{c:32s} {tot[c] / max(1, len(disp[c])):16.1f}")
