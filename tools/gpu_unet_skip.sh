# Phase-skip experiment on the U-Net convs (timing only; results are garbage): which phase is on the
# critical path. Fixed model-picked tiling (no autotune), non-persistent kernels.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/unet_skip.log
: > $L
for dt in f16 f32x3; do
  for sk in 0 1 2 4 8 5 13 14 15; do
    echo "skip=$sk" >> $L
    MPCD_UNET_AUTOTUNE=0 MPCD_UNET_SKIP=$sk timeout -k 10 120 python tools/unet_perf.py --B 16384 --H 32 --C 2 --steps 4 --reps 1 --dtype $dt >> $L 2>&1 || exit $?
  done
done
