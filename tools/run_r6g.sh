# round 6: Linear 8's loads split over Linear 5 / 6 (w8s) against the product (early cond tables); per-layer profile
cd $GRAFT_REPO_ROOT
export BENCH_ARGS="--no-shard-probe"
bash tools/gpu.sh bench:cfg2 mlpab:w8s || exit $?
bash tools/mlp_prof.sh 4096
