"""Per-shape A/B table from interleaved kernel-timing logs (lines "TAG <shape>: <us> us ..."):
the mean of each arm's runs per shape and B / A.
    python tools/ab_table.py LOG [A_TAG] [B_TAG]"""
import collections
import re
import sys

path = sys.argv[1]
ta = sys.argv[2] if len(sys.argv) > 2 else "cur"
tb = sys.argv[3] if len(sys.argv) > 3 else "B"
t = collections.defaultdict(lambda: collections.defaultdict(list))
order = []
for line in open(path):
    m = re.match(r"(\S+) (.*?):\s+([\d.]+) us", line)
    if not m:
        continue
    tag, shape, us = m.group(1), m.group(2), float(m.group(3))
    if shape not in order:
        order.append(shape)
    t[shape][tag].append(us)
sa = sb = 0.0
for s in order:
    a, b = t[s].get(ta, []), t[s].get(tb, [])
    if not a or not b:
        continue
    ma, mb = sum(a) / len(a), sum(b) / len(b)
    sa += ma
    sb += mb
    print(f"{s:45s} A {ma:8.1f}  B {mb:8.1f}  B/A {mb / ma:5.3f}")
if sa:
    print(f"{'total':45s} A {sa:8.1f}  B {sb:8.1f}  B/A {sb / sa:5.3f}")
