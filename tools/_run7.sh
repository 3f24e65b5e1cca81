set -o pipefail
export MPCD_SPREAD_LOG=$PWD/gpurun_out/spread_ratios.tsv
timeout -k 10 500 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_unet_fused.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_mlp_fused.log 2>&1
echo "pytest rc=$?" >> gpurun_out/t_mlp_fused.log; tail -3 gpurun_out/t_mlp_fused.log
timeout -k 10 300 python -u bench.py --workload cfg2 --no-cpu-baseline > gpurun_out/b_base.log 2>&1 || exit 1
MPCD_MLP_LAYOUT=rw32 timeout -k 10 300 python -u bench.py --workload cfg2 --no-cpu-baseline --no-shard-probe > gpurun_out/b_rw32.log 2>&1 || exit 1
MPCD_MLP_LAYOUT=rw16 timeout -k 10 300 python -u bench.py --workload cfg2 --no-cpu-baseline > gpurun_out/b_rw16.log 2>&1 || exit 1
for c in cfg3 cfg5; do bash tools/gpu.sh unet:$c || exit 1; done
MPCD_FUSED_PERSIST=1 timeout -k 10 600 python -u tools/unet_perf.py --B 16384 --H 32 --d 1 --C 2 --N 100 --dtype f32x3 > gpurun_out/unet_cfg3_persist.log 2>&1 || exit 1
MPCD_FUSED_PERSIST=1 timeout -k 10 600 python -u tools/unet_perf.py --B 65536 --H 64 --d 1 --C 5 --N 100 --dtype f32x3 > gpurun_out/unet_cfg4_persist.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/unet_perf.py --B 65536 --H 64 --d 1 --C 5 --N 100 --dtype f32x3 > gpurun_out/unet_cfg4.log 2>&1 || exit 1
tail -2 gpurun_out/unet_*.log
