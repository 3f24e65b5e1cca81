# round 6: packed exposed last-pass epilogue (pk) against the product, alternating, and the MLP parity of pk
cd $GRAFT_REPO_ROOT
export BENCH_ARGS="--no-shard-probe"
MPCD_LIB=$PWD/mpc_via_diffusion_model_amd/libmpcd_pk.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py \
  tests/test_gpu_headline.py tests/test_gpu_mlp_h2.py tests/test_gpu_rollout.py tests/test_golden.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pk.log 2>&1 || { echo "pytest pk failed"; tail -n 30 gpurun_out/pytest_pk.log; exit 1; }
tail -n 1 gpurun_out/pytest_pk.log
for r in 1 2 3; do
  bash tools/gpu.sh bench:cfg2 mlpab:pk || exit $?
  for f in gpurun_out/bench_cfg2.log gpurun_out/mlpab_pk.log; do
    python -c "import json; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('rep $r $f', round(d['value']), d['ms_per_step'], d['roofline'].get('kernel_ms'))"
  done
done
