"""HBM traffic per launch of one kernel from two rocprofv3 counter passes (FETCH_SIZE and
WRITE_SIZE, separate runs), with the gfx950 correction of MI355X_MICROARCH.md (HBM /
rocprofv3 section): FETCH_SIZE counts half the bytes of 16-B-per-lane streaming reads, so it
is doubled; WRITE_SIZE is exact for 16-B stores.  Both counters are in KiB.

    python tools/pmc_json.py FILTER fetch_counter_collection.csv write_counter_collection.csv OUT.json
"""
import csv
import json
import sys
from collections import defaultdict


def per_dispatch(path, flt, counter):
    vals = defaultdict(float)
    for row in csv.DictReader(open(path)):
        if flt in row["Kernel_Name"] and row["Counter_Name"] == counter:
            vals[row["Dispatch_Id"]] += float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for kernels matching {flt!r} in {path}")
    return sum(vals.values()) / len(vals), len(vals)


def main():
    flt, fetch_csv, write_csv, out = sys.argv[1:5]
    fetch_kib, n_f = per_dispatch(fetch_csv, flt, "FETCH_SIZE")
    write_kib, n_w = per_dispatch(write_csv, flt, "WRITE_SIZE")
    read_b = 2.0 * fetch_kib * 1024.0
    write_b = write_kib * 1024.0
    res = {"kernel_filter": flt, "dispatches": [n_f, n_w],
           "fetch_size_kib": round(fetch_kib, 1), "write_size_kib": round(write_kib, 1),
           "read_bytes_corrected": int(read_b), "write_bytes": int(write_b),
           "hbm_bytes_per_launch": int(read_b + write_b),
           "note": "read = 2 x FETCH_SIZE (gfx950 correction), write = WRITE_SIZE; separate --pmc passes"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
