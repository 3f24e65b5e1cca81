# fp16 activation buffers for the f16 U-Net: parity, then throughput with / without (MPCD_UNET_F16_ACT)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/f16act
timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/f16act/pytest_unet.log 2>&1 || exit $?
L=gpurun_out/f16act/perf.log
: > $L
for act in 0 1; do
  MPCD_UNET_F16_ACT=$act timeout -k 10 200 python tools/unet_perf.py --B 16384 --H 32 --d 1 --C 2 --steps 10 --dtype f16 >> $L 2>&1 || exit $?
  MPCD_UNET_F16_ACT=$act timeout -k 10 200 python tools/unet_perf.py --B 16384 --H 64 --d 4 --C 12 --N 250 --schedule cosine --steps 5 --dtype f16 >> $L 2>&1 || exit $?
done
