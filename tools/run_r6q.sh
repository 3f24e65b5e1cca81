# round 6 (second session) closing run (b) on the final build: GPU suite (spread ratios logged), smoke, every workload's
# bench line (cfg1-5 with same-build traffic), Panda (the reference's published timing) and the opt-in f16x2 cfg2 line
cd $GRAFT_REPO_ROOT
export MPCD_SPREAD_LOG=$PWD/gpurun_out/spread_ratios.tsv
rm -f "$MPCD_SPREAD_LOG"
bash tools/gpu.sh tests smoke bench:cfg2 bench:cfg1 bench:cfg3 bench:cfg4 bench:cfg5 || exit $?
timeout -k 10 300 python -u bench.py --workload panda > gpurun_out/bench_panda.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload cfg2 --dtype f16x2 > gpurun_out/bench_cfg2_f16x2.log 2>&1
