# Kernel-trace timing of the window-attention kernels at one shape, dropout off and on:
#   bash tools/attn_time.sh TAG res nh shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/attn_time_$TAG
mkdir -p $O
for p in 0.0 0.05; do
  timeout -k 10 60 rocprofv3 --kernel-trace --stats -d $O -o kt_$p --output-format csv -- python3 $R/tools/attn_one.py $1 $2 $3 1 5 $p > $O/kt_$p.log 2>&1 || { tail -5 $O/kt_$p.log; exit 1; }
  python3 - $O/kt_${p}_kernel_stats.csv $p <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'attn' in r['Name']:
        print(sys.argv[2], r['Name'].split('(')[0][-40:], r['Name'].split('<')[1].split('>')[0], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
done
