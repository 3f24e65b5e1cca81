# round 6: the MLP sampler's timing events recorded by its launch (hipExtLaunchKernel) against separate
# hipEventRecord calls around it (libmpcd_sepev.so, -DMPCD_SEPARATE_EVENT_RECORDS=1), alternating on one box
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_headline.py tests/test_gpu_rollout.py \
  tests/test_gpu_mlp_h2.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_ev.log 2>&1 || { echo "pytest failed"; tail -n 30 gpurun_out/pytest_ev.log; exit 1; }
tail -n 1 gpurun_out/pytest_ev.log
for r in 1 2 3; do
  for v in ext sep; do
    for w in cfg2 cfg1; do
      if [ $v = sep ]; then export MPCD_LIB=$PWD/mpc_via_diffusion_model_amd/libmpcd_sepev.so; else unset MPCD_LIB; fi
      timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-shard-probe > gpurun_out/ab_${v}_$w.log 2>&1 || exit 1
      python -c "import json; l=[x for x in open('gpurun_out/ab_${v}_$w.log') if x.startswith('{')][-1]; d=json.loads(l); print('rep $r $v $w', round(d['value']), round(d['ms_per_step'], 4), round(d['roofline']['kernel_ms'], 4))"
    done
  done
done
