set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export MPCD_SPREAD_LOG=$PWD/gpurun_out/spread.tsv
rm -f $MPCD_SPREAD_LOG
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp_h2.py tests/test_gpu_headline.py -x -v -s --timeout 240 --timeout-method thread > gpurun_out/h2tests.log 2>&1
rc=$?; echo "h2tests rc=$rc" >> gpurun_out/h2tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --dtype f16x2 --no-cpu-baseline > gpurun_out/bench_h2.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --dtype f32x3 --no-cpu-baseline > gpurun_out/bench_x3.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_bench_launch.py -x -v --timeout 280 --timeout-method thread > gpurun_out/launch.log 2>&1; echo "launch rc=$?" >> gpurun_out/launch.log
bash tools/gpu.sh tests
