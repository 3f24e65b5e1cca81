# U-Net: parity tests, then throughput at the BASELINE U-Net shapes (autotuned conv tiling).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_unet.log 2>&1 || exit $?
L=gpurun_out/unet_perf.log
: > $L
for dt in f16 f32x3; do
  timeout -k 10 200 python tools/unet_perf.py --B 16384 --H 32 --d 1 --C 2 --steps 10 --dtype $dt >> $L 2>&1 || exit $?
  timeout -k 10 200 python tools/unet_perf.py --B 8192 --H 64 --d 1 --C 5 --steps 5 --dtype $dt >> $L 2>&1 || exit $?
  timeout -k 10 200 python tools/unet_perf.py --B 16384 --H 64 --d 4 --C 12 --N 250 --schedule cosine --steps 5 --dtype $dt >> $L 2>&1 || exit $?
done
