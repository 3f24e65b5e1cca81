# Phase-skip experiment at the cfg5 shape (f16, B=131072 candidates, H=64, d=4, C=12): timing only,
# results are garbage. skip bits: 1 staging, 2 GEMM, 4 GroupNorm statistics, 8 epilogue.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/unet_skip5.log
: > $L
for sk in 0 1 2 4 8 14 13 11 7 15; do
  echo "skip=$sk" >> $L
  MPCD_UNET_AUTOTUNE=0 MPCD_UNET_SKIP=$sk timeout -k 10 120 python tools/unet_perf.py --B 131072 --H 64 --d 4 --C 12 --steps 3 --reps 1 --dtype f16 --schedule cosine --N 250 --fuse 0 >> $L 2>&1 || exit $?
done
