# Profile the headline bench: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in separate passes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run -f csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof/trace_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex mlp_sample -d gpurun_out/prof/fetch -o run -f csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex mlp_sample -d gpurun_out/prof/write -o run -f csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex mlp_sample -d gpurun_out/prof/sq -o run -f csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/sq.log 2>&1
find gpurun_out/prof -name "*.csv" | head -50
