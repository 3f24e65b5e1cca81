# cfg5-shape forward time vs the first-generation stagger (tuned tilings from profiles/, unfused convs)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/unet_stagger.log
: > $L
cp profiles/r2_unet_tune_cfg5.txt /tmp/tune5.txt
for st in 0 2 4 8 16 0; do
  echo "stagger=$st" >> $L
  MPCD_UNET_TUNE_CACHE=/tmp/tune5.txt MPCD_UNET_STAGGER=$st timeout -k 10 120 python tools/unet_perf.py --B 131072 --H 64 --d 4 --C 12 --steps 3 --reps 2 --dtype f16 --schedule cosine --N 250 --fuse 0 >> $L 2>&1 || exit $?
done
