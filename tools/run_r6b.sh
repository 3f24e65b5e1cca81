# round 6: the f32x3 cfg2 line, GPU suite (spread ratios logged), SQ counters, per-layer profile
cd $GRAFT_REPO_ROOT
export MPCD_SPREAD_LOG=$PWD/gpurun_out/spread_ratios.tsv
rm -f "$MPCD_SPREAD_LOG"
bash tools/gpu.sh bench:cfg2 tests sqpmc:4096 || exit $?
bash tools/mlp_prof.sh 4096 512
