# Kernel-trace a kbench mode: bash tools/prof_kbench.sh MODE [ENV=VAL ...]; writes gpurun_out/pk_MODE/
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
M=$1; shift
for kv in "$@"; do export "$kv"; done
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pk_$M -o run -- python3 -u $R/tools/kbench.py $M > $R/gpurun_out/pk_$M.log 2>&1
cat $R/gpurun_out/pk_$M.log | grep -v Warning
f=$(find $R/gpurun_out/pk_$M -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:25]:
    print(f"{float(r['AverageNs'])/1e3:9.1f} us x{int(r['Calls']):4d}  {r['Name'][:150]}")
PY
