# Every BASELINE workload through bench.py on one GPU (cfg4 / cfg5 at N = 1 carry the whole batch).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in cfg2 cfg1 cfg3 cfg4 cfg5; do
  timeout -k 10 300 python -u bench.py --workload $w --cpu-budget 10 > gpurun_out/bench_$w.log 2>&1 || exit $?
done
