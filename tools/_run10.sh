set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_mlp.py tests/test_gpu_comm.py tests/test_gpu_multiprocess.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_r10.log 2>&1; rc=$?; tail -2 gpurun_out/t_r10.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_cfg2_final.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload cfg1 > gpurun_out/bench_cfg1_final.log 2>&1 || exit 1
bash tools/gpu.sh trace:cfg2 pmc:cfg2 || exit 1
tail -c 400 gpurun_out/bench_cfg2_final.log
