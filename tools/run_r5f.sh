# round 5: two-term fp16 fused U-Net (P = 2) - parity at small and bench sizes, then the cfg4 / panda lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_unet_fused.py tests/test_gpu_unet.py tests/test_gpu_unet_bench_sizes.py -x -v -s -rs --timeout 400 --timeout-method thread -k "h128 or panda or fused or h2" > gpurun_out/unet_h2_tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/unet_h2_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --workload panda --dtype f16x2 --steps 100 > gpurun_out/bench_panda_f16x2.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --workload cfg4 --dtype f16x2 --no-cpu-baseline > gpurun_out/bench_cfg4_h2.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --workload cfg4 --dtype f32x3 --no-cpu-baseline > gpurun_out/bench_cfg4_x3.log 2>&1
