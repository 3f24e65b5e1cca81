# Round-2 headline evidence: rocprofv3 kernel-trace stats of the default bench command (cfg2) and the
# FETCH_SIZE / WRITE_SIZE passes of its sampler kernel (one counter per pass, kernel trace only)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2/trace -o run -f csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof2/trace_bench.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "mlp_x3_kernel" -d gpurun_out/prof2/$c -o run -f csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof2/$c.log 2>&1 || exit $?
done
