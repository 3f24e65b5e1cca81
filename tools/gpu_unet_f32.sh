cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py tests/test_golden.py -q --timeout 150 --timeout-method thread > gpurun_out/unet_f32_tests.log 2>&1 || exit 1
for i in 1 2; do timeout -k 10 200 python tools/unet_perf.py --B 4096 --H 32 --d 1 --C 2 --steps 3 --reps 1 --dtype f32 >> gpurun_out/unet_f32_perf.log 2>&1 || exit 1; done
