"""The bench's roofline launches in a rocprofv3 kernel trace of the bench command: the longest run
of back-to-back launches of one kernel (conv_roofline: 3 warmup + 10 timed launches of the
refine2 forward), its average duration over the timed ones, beside the bench line's
``roofline.ms_per_launch`` from the same run.

    python tools/roofline_trace.py TRACE.csv BENCH.json [KERNEL_SUBSTRING]"""
import csv
import json
import sys


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    sub = sys.argv[3] if len(sys.argv) > 3 else "conv3x3_v3_kernel<unsigned short, false, false, false, true, false, true, true>"
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    best, run = [], []
    for r in rows:
        if sub in r["Kernel_Name"]:
            run.append(r)
            if len(run) > len(best):
                best = list(run)
        else:
            run = []
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in best]
    timed = d[-10:]
    line = next(json.loads(ln) for ln in open(bench) if ln.startswith("{"))
    print(f"kernel: {sub}")
    print(f"longest back-to-back run: {len(d)} launches; ms per launch: {' '.join(f'{x:.4f}' for x in d)}")
    print(f"trace average over the last {len(timed)}: {sum(timed) / len(timed):.4f} ms")
    print(f"bench roofline.ms_per_launch (HIP events, same run): {line['roofline']['ms_per_launch']:.4f} ms")


if __name__ == "__main__":
    main()
