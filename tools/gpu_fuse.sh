# Fused ResidualTemporalBlock: U-Net parity (incl. fused vs unfused bit identity), then throughput
# with the fused launch never / always / measured, at cfg3 and cfg4-shard shapes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/fuse
timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fuse/pytest_unet.log 2>&1 || exit $?
L=gpurun_out/fuse/perf.log
: > $L
for dt in f16 f32x3; do
  for fu in 0 1 ""; do
    timeout -k 10 200 python tools/unet_perf.py --B 16384 --H 32 --d 1 --C 2 --steps 10 --dtype $dt --fuse "$fu" >> $L 2>&1 || exit $?
  done
  for fu in 0 ""; do
    timeout -k 10 200 python tools/unet_perf.py --B 8192 --H 64 --d 1 --C 5 --steps 5 --dtype $dt --fuse "$fu" >> $L 2>&1 || exit $?
  done
done
