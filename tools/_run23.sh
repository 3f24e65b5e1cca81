set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_headline.py tests/test_gpu_rollout.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r23_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r23_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 300 python -u bench.py --workload cfg2 --no-cpu-baseline > gpurun_out/r23_cfg2_$i.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r23_cfg2_$i.log | tr '\n' ' '; echo; done
timeout -k 10 300 python -u bench.py --workload cfg1 --no-cpu-baseline > gpurun_out/r23_cfg1.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r23_cfg1.log | tr '\n' ' '; echo
