# MLP x3 workgroup layouts: parity probe, then cfg1 / cfg2 bench under each forced layout
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=gpurun_out/mlp_layouts.log
: > $L
timeout -k 10 200 python -u tools/diag_rows16.py >> $L 2>&1 || exit $?
for lay in 32x8 16x8 16x4; do
  for w in cfg2 cfg1; do
    echo "layout=$lay $w" >> $L
    MPCD_MLP_LAYOUT=$lay timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/lay_${lay}_$w.json 2>> $L || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'], (d.get('strong_shard_probe') or {}).get('ms_per_step'))" gpurun_out/lay_${lay}_$w.json >> $L
  done
done
