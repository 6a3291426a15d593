#!/bin/bash
# A/B of the HIP-graph replay against the eager step (and HIP graph runtime settings).
# usage (GPU box): bash tools/graph_ab.sh [extra bench args]
mkdir -p gpurun_out/ab
run() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-input-pipeline $BENCH_ARGS \
    > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.err || { echo "$name FAILED"; tail -3 gpurun_out/ab/$name.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/$name.json'));print('$name', d['value'], d['ms_per_step'], d['host_ms_per_step'], d['config']['step_execution'])"
}
