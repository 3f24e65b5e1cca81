set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_headline.py tests/test_gpu_multiprocess.py tests/test_gpu_rollout.py tests/test_gpu_trained_lmpc.py tests/test_gpu_closed_loop.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r17_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r17_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload cfg2 --no-cpu-baseline > gpurun_out/r17_cfg2.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/host_overhead.py 4096 > gpurun_out/r17_host.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r17_cfg2.log | tr '\n' ' '; echo; head -2 gpurun_out/r17_host.log
