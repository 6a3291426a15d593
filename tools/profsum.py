import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
steps=float(sys.argv[2]) if len(sys.argv)>2 else 1
tot=sum(float(r['TotalDurationNs']) for r in rows)
print(f"total {tot/1e6:.1f} ms  per-step {tot/1e6/steps:.1f} ms  kernels {len(rows)}")
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv)>3 else 30]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.2f} ms/step {float(r['Percentage']):5.1f}% n={int(r['Calls'])/steps:6.1f} avg={float(r['AverageNs'])/1e3:8.1f}us {r['Name'][:100]}")
