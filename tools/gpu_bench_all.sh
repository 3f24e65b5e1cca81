#!/bin/bash
# GPU box: every BASELINE workload through bench.py (one JSON line each) into gpurun_out/bench_<cfg>.json.
# usage: bash tools/gpu_bench_all.sh [cfg...]   (default: all five)
set -o pipefail
mkdir -p gpurun_out
cfgs=${@:-cfg2 cfg1 cfg3 cfg4 cfg5}
for w in $cfgs; do
  timeout -k 10 400 python -u bench.py --workload $w > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { echo "bench $w failed"; exit 1; }
  tail -c 400 gpurun_out/bench_$w.json
done
