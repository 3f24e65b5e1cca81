# round 6: per-layer profile of the final build (MPCD_PROF_LAYERS) and the update's cost as a bound (nu: the final
# layer's MFMAs without the update, wrong results) against the product
cd $GRAFT_REPO_ROOT
export BENCH_ARGS="--no-shard-probe"
bash tools/mlp_prof.sh 4096 512 || exit $?
bash tools/gpu.sh bench:cfg2 mlpab:nu || exit $?
for f in gpurun_out/bench_cfg2.log gpurun_out/mlpab_nu.log; do
  python -c "import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f', round(d['value']), d['ms_per_step'], d['roofline'].get('kernel_ms'))"
done
