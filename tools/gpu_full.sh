# Full GPU pass: parity tests, smoke, bench (both GEMM numerics), rocprofv3 kernel-trace stats of the
# headline bench and FETCH_SIZE / WRITE_SIZE passes (one counter block per pass) for the MLP kernels.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
rocminfo 2>/dev/null | grep -m2 -E "gfx950|Marketing" > gpurun_out/rocminfo.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dtype f32 > gpurun_out/bench_f32.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run -f csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof/trace_bench.log 2>&1 || exit $?
for dt in f32x3 f32; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "mlp_(x3|sample)_kernel" -d gpurun_out/prof/${dt}_$c -o run -f csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --dtype $dt > gpurun_out/prof/${dt}_$c.log 2>&1 || exit $?
  done
done
find gpurun_out/prof -name "*.csv" > gpurun_out/prof/files.txt
