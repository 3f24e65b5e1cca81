# U-Net throughput at the BASELINE U-Net shapes (per-GPU shards) for every GEMM numerics, then a
# rocprofv3 kernel-trace of the cfg3 run.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_unet
L=gpurun_out/unet_perf.log
: > $L
for dt in f16; do
  timeout -k 10 200 python tools/unet_perf.py --B 16384 --H 32 --d 1 --C 2 --steps 10 --dtype $dt >> $L 2>&1 || exit $?
done
for dt in f16 f32x3; do
  timeout -k 10 200 python tools/unet_perf.py --B 8192 --H 64 --d 1 --C 5 --steps 5 --dtype $dt >> $L 2>&1 || exit $?
  timeout -k 10 200 python tools/unet_perf.py --B 16384 --H 64 --d 4 --C 12 --N 250 --schedule cosine --steps 5 --dtype $dt >> $L 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_unet -o run -f csv -- python3 tools/unet_perf.py --B 16384 --H 32 --C 2 --steps 4 --reps 1 > gpurun_out/prof_unet/log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_unet_f16 -o run -f csv -- python3 tools/unet_perf.py --B 16384 --H 32 --C 2 --steps 4 --reps 1 --dtype f16 > gpurun_out/prof_unet_f16.log 2>&1
