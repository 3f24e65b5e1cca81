# round 6 closing run (a) on the committed build: GPU suite (spread ratios logged), smoke, the cfg2 headline line, its
# rocprofv3 kernel trace, FETCH/WRITE passes for cfg2 and cfg1, SQ counters of the headline kernel
cd $GRAFT_REPO_ROOT
export MPCD_SPREAD_LOG=$PWD/gpurun_out/spread_ratios.tsv
rm -f "$MPCD_SPREAD_LOG"
bash tools/gpu.sh bench:cfg2 smoke tests || exit $?
bash tools/gpu.sh trace:cfg2 pmc:cfg2 pmc:cfg1 sqpmc:4096
