# A/B of two libmpcd builds on the MLP workloads (kernel ms from bench.py), then the MLP GPU tests
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=gpurun_out/mlp_ab.log
: > $L
for rep in 1 2; do
for lib in libmpcd.so ${ALT:-libmpcd_noilv.so}; do
  for w in cfg2 cfg1; do
    echo "$lib $w" >> $L
    MPCD_LIB=mpc_via_diffusion_model_amd/$lib timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/ab.json 2>> $L || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'], (d.get('strong_shard_probe') or {}).get('ms_per_step'))" gpurun_out/ab.json >> $L
  done
done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread >> $L 2>&1
