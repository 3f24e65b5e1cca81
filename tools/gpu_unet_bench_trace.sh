# Kernel-trace stats of the U-Net bench workloads themselves (cfg3 f32x3, cfg5 f16), one timed step each.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in cfg3 cfg5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/btr_$w -o run -f csv -- python3 bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/btr_$w.log 2>&1 || exit $?
done
