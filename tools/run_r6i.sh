# round 6: repeat of product vs tsxr (alternating order) to separate the difference from run-to-run noise
cd $GRAFT_REPO_ROOT
export BENCH_ARGS="--no-shard-probe"
for r in 1 2 3; do
  bash tools/gpu.sh bench:cfg2 mlpab:tsxr || exit $?
  for f in gpurun_out/bench_cfg2.log gpurun_out/mlpab_tsxr.log; do
    python -c "import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('rep $r $f', round(d['value']), d['ms_per_step'], d['roofline'].get('kernel_ms'))"
  done
done
