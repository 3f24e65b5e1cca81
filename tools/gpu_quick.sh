# Quick GPU pass: the rollout / comm / MLP parity tests, then the default bench (no CPU baseline).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_comm.py tests/test_gpu_closed_loop.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --warmup 10 >> gpurun_out/bench_quick.log 2>&1 || exit $?
