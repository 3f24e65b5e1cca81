# cfg5-shape forward time per candidate vs batch (does a batch that fits the 256 MB Infinity Cache run faster?)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/unet_bsweep.log
: > $L
for b in 2048 8192 32768 131072; do
  timeout -k 10 200 python tools/unet_perf.py --B $b --H 64 --d 4 --C 12 --steps 3 --reps 2 --dtype f16 --schedule cosine --N 250 >> $L 2>&1 || exit $?
done
