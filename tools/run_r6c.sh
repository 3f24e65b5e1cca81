# round 6: SQ counters and per-layer profile of the f32x3 MLP kernel first, then the GPU suite (spread ratios logged)
cd $GRAFT_REPO_ROOT
export MPCD_SPREAD_LOG=$PWD/gpurun_out/spread_ratios.tsv
rm -f "$MPCD_SPREAD_LOG"
bash tools/gpu.sh sqpmc:4096 || exit $?
bash tools/mlp_prof.sh 4096 512 || exit $?
bash tools/gpu.sh tests
