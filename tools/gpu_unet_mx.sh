# U-Net mx kernels + comm: parity tests, then throughput per GEMM numerics (+ kernel-trace of the x3 run)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_unet_mx
timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_comm.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_unet.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_unet.log; if [ $rc -gt 1 ]; then exit $rc; fi
for dt in f32x3 f16; do
  timeout -k 10 200 python tools/unet_perf.py --B 16384 --H 32 --C 2 --steps 10 --dtype $dt >> gpurun_out/unet_perf.log 2>&1 || exit $?
  timeout -k 10 200 python tools/unet_perf.py --B 8192 --H 64 --C 5 --steps 5 --dtype $dt >> gpurun_out/unet_perf.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_unet_mx -o run -f csv -- python3 tools/unet_perf.py --B 16384 --H 32 --C 2 --steps 4 --reps 1 --dtype f32x3 > gpurun_out/prof_unet_mx/log 2>&1
