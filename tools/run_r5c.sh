# round 5: fused fp32-accurate Panda (unet_fused_kernel<3, 1, 128, 8>) - parity, then the published-config timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet_fused.py tests/test_gpu_unet.py -x -v -s -rs --timeout 300 --timeout-method thread -k "h128 or panda" > gpurun_out/panda_tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/panda_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --workload panda --dtype f32x3 --steps 100 > gpurun_out/bench_panda_f32x3.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload panda --dtype f16 --steps 100 > gpurun_out/bench_panda_f16.log 2>&1
