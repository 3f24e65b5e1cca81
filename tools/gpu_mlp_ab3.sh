# A/B/C of libmpcd builds on cfg2 / cfg1 (kernel ms from bench.py)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=gpurun_out/mlp_ab3.log
: > $L
for rep in 1 2; do
for lib in libmpcd.so $ALTS; do
  for w in cfg2 cfg1; do
    MPCD_LIB=mpc_via_diffusion_model_amd/$lib timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/ab.json 2>> gpurun_out/ab.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], 'kernel_ms %.4f' % d['roofline']['kernel_ms'], 'step_ms %.4f' % d['ms_per_step'], 'frac %.4f' % d['roofline']['frac'], 'shard_ms', (d.get('strong_shard_probe') or {}).get('ms_per_step'))" gpurun_out/ab.json $lib $w >> $L
  done
done
done
