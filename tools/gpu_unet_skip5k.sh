# Phase-skip timing at the cfg5 shape with the bench's tuned tilings (profiles/r2_unet_tune_cfg5.txt) kept
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/unet_skip5k.log
: > $L
cp profiles/r2_unet_tune_cfg5.txt /tmp/tune5.txt
for sk in 0 1 2 4 8 14 13 11 7 15; do
  echo "skip=$sk" >> $L
  MPCD_UNET_TUNE_CACHE=/tmp/tune5.txt MPCD_UNET_SKIP_KEEP=1 MPCD_UNET_SKIP=$sk timeout -k 10 120 python tools/unet_perf.py --B 131072 --H 64 --d 4 --C 12 --steps 3 --reps 1 --dtype f16 --schedule cosine --N 250 --fuse 0 >> $L 2>&1 || exit $?
done
