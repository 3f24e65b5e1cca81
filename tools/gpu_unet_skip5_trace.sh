# Kernel trace of the cfg5-shape probe with every conv phase skipped (what is left outside the convs)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for sk in 15 0; do
  MPCD_UNET_AUTOTUNE=0 MPCD_UNET_SKIP=$sk timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/skip5tr_$sk -o run -- python tools/unet_perf.py --B 131072 --H 64 --d 4 --C 12 --steps 3 --reps 1 --dtype f16 --schedule cosine --N 250 > gpurun_out/skip5tr_$sk.log 2>&1 || exit $?
done
