# Phase-skip timing at the cfg3 shape (f32x3, B=16384, H=32, d=1, C=2), tuned tilings kept; timing only
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/unet_skip3k.log
: > $L
cp profiles/r2_unet_tune_cfg3.txt /tmp/tune3.txt
for sk in 0 14 13 11 7 15; do
  echo "skip=$sk" >> $L
  MPCD_UNET_TUNE_CACHE=/tmp/tune3.txt MPCD_UNET_SKIP_KEEP=1 MPCD_UNET_SKIP=$sk timeout -k 10 120 python tools/unet_perf.py --B 16384 --H 32 --d 1 --C 2 --steps 4 --reps 1 --dtype f32x3 --fuse 0 >> $L 2>&1 || exit $?
done
