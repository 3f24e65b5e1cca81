# round 6: the fused control-step tail (an experiment, reverted: profiles/r6_mlp_tail_ab.txt) against the separate rollout launch
# alternating on one box, cfg2 and cfg1; parity of the tail first
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_headline.py tests/test_gpu_mlp.py \
  tests/test_gpu_closed_loop.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_tail.log 2>&1 || { echo "pytest failed"; tail -n 30 gpurun_out/pytest_tail.log; exit 1; }
tail -n 1 gpurun_out/pytest_tail.log
for r in 1 2 3; do
  for mode in tail sep; do
    for w in cfg2 cfg1; do
      if [ $mode = sep ]; then export MPCD_NO_FUSED_TAIL=1; else unset MPCD_NO_FUSED_TAIL; fi
      timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-shard-probe > gpurun_out/ab_${mode}_$w.log 2>&1 || exit 1
      python -c "import json; l=[x for x in open('gpurun_out/ab_${mode}_$w.log') if x.startswith('{')][-1]; d=json.loads(l); print('rep $r $mode $w', round(d['value']), round(d['ms_per_step'], 4), round(d['roofline']['kernel_ms'], 4))"
    done
  done
done
