set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_headline.py tests/test_gpu_closed_loop.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r26_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r26_tests.log
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace26 -o run -f csv -- python3 bench.py --workload cfg2 --no-cpu-baseline --no-shard-probe > gpurun_out/r26_trace.log 2>&1 || exit 1
python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/prof/trace26/run_kernel_stats.csv')))[:4]: print(r['Name'][:50], r['AverageNs'])"
