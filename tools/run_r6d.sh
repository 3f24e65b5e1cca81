# round 6: split-bf16 MLP kernel with per-column-tile counters (product) vs the barrier form (libmpcd_bar.so)
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh "tests:mlp or headline or rollout or closed" bench:cfg2 mlpab:bar
