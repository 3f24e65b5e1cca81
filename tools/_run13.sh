set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_headline.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r13_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r13_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload cfg2 --no-cpu-baseline > gpurun_out/r13_cfg2.log 2>&1 || exit 1
bash tools/gpu.sh mlpab:nodefer || exit 1
for f in r13_cfg2 mlpab_nodefer; do grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/$f.log | tr '\n' ' '; echo; done
