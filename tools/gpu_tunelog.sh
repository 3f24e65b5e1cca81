# U-Net autotune log (every measured candidate) at the cfg3 shape, both numerics
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rx
for dt in f16 f32x3; do
  MPCD_UNET_TUNE_LOG=1 timeout -k 10 200 python tools/unet_perf.py --B 16384 --H 32 --d 1 --C 2 --steps 10 --dtype $dt > gpurun_out/rx/tune_$dt.log 2>&1 || exit $?
done
