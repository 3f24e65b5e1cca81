# round 6: product (Linear 8 loads split over Linear 5 / 6) against the Linear-12 side-work table (ts), x_t in
# registers with the update's x-only products hoisted (xr), and both (tsxr); MLP parity of each
cd $GRAFT_REPO_ROOT
export BENCH_ARGS="--no-shard-probe"
bash tools/gpu.sh bench:cfg2 mlpab:ts mlpab:xr mlpab:tsxr || exit $?
bash tools/gpu.sh "tests:mlp or headline" || exit $?
for v in ts xr tsxr; do
  MPCD_LIB=$PWD/mpc_via_diffusion_model_amd/libmpcd_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py \
    tests/test_gpu_headline.py tests/test_gpu_mlp_h2.py tests/test_gpu_rollout.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$v.log 2>&1 || { echo "pytest $v failed"; exit 1; }
done
for f in gpurun_out/bench_cfg2.log gpurun_out/mlpab_*.log; do
  python -c "import json,sys; l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l); print('$f', round(d['value']), d['ms_per_step'], d['roofline'].get('kernel_ms'))"
done
