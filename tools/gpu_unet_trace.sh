# Kernel traces of the U-Net sampler (cfg3 shape) for both mx numerics; per-layer tables come from
# tools/unet_layer_table.py on the last forward of each trace.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for dt in f16 f32x3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$dt -o run -f csv -- python3 tools/unet_perf.py --B 16384 --H 32 --C 2 --steps 4 --reps 1 --dtype $dt > gpurun_out/tr_$dt.log 2>&1 || exit $?
done
