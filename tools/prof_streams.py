"""Per-stream kernel-time summary of a rocprofv3 --kernel-trace CSV (the eager step's main and
side streams): kernel ms per step on each stream and its top kernels by time.

    python tools/prof_streams.py gpurun_out/TAG_prof/p_kernel_trace.csv STEPS [TOP]

STEPS = warmup + timed steps of the profiled bench run (every step is traced)."""
import collections
import csv
import re
import sys


def short(name, grid, wg):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "").replace("unsigned short", "u16")
    n = re.split(r"\((?!anon)", n)[0][:80]
    return f"{n} [{int(grid) // max(1, int(wg))} wg]"


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows = list(csv.DictReader(open(path)))
    by_stream = collections.defaultdict(list)
    for r in rows:
        by_stream[r["Stream_Id"]].append(r)
    t0 = min(int(r["Start_Timestamp"]) for r in rows)
    t1 = max(int(r["End_Timestamp"]) for r in rows)
    print(f"trace span {(t1 - t0) / 1e6 / steps:.2f} ms per step over {steps} steps; {len(rows)} launches")
    for sid, rs in sorted(by_stream.items(), key=lambda kv: -len(kv[1])):
        t = collections.defaultdict(float)
        c = collections.Counter()
        for r in rs:
            k = short(r["Kernel_Name"], r["Grid_Size_X"], r["Workgroup_Size_X"])
            t[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 / steps
            c[k] += 1
        print(f"\n== stream {sid}: {sum(t.values()):.2f} ms of kernel time per step, {len(rs) / steps:.0f} launches per step")
        print(" ms/step  n/step   avg us  kernel")
        for k, v in sorted(t.items(), key=lambda kv: -kv[1])[:top]:
            n = c[k] / steps
            print(f"{v:8.3f} {n:7.1f} {1e3 * v / n:8.1f}  {k}")


if __name__ == "__main__":
    main()
