# round 5: the fused U-Net with swizzled positions - parity, then cfg5 / cfg4 / cfg3 timing and LDS counters
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/uroof
timeout -k 10 900 python -u -m pytest tests/test_gpu_unet_fused.py tests/test_gpu_unet.py tests/test_gpu_unet_bench_sizes.py tests/test_gpu_trained_lmpc.py -x -q --timeout 400 --timeout-method thread > gpurun_out/unet_swz_tests.log 2>&1 || exit $?
for c in cfg5 cfg4h cfg3; do
  true
done
timeout -k 10 300 python -u tools/unet_perf.py --B 131072 --H 64 --d 4 --C 12 --N 250 --schedule cosine --sampler ddpm_cfg --dtype f16 --reps 1 > gpurun_out/unet_swz_cfg5.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/unet_perf.py --B 65536 --H 64 --d 1 --C 5 --N 100 --sampler ddpm_cfg --dtype f16x2 --reps 1 > gpurun_out/unet_swz_cfg4.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/unet_perf.py --B 16384 --H 32 --d 1 --C 2 --N 100 --steps 100 --dtype f32x3 --reps 2 > gpurun_out/unet_swz_cfg3.log 2>&1 || exit $?
bash tools/run_r5l.sh
