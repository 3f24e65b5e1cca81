# round 6 closing run (b) on the committed build: the other workloads' lines (cfg1, cfg3, cfg4, cfg5, Panda) and the
# opt-in two-term fp16 cfg2 line; cfg2 again first, now that the PMC summaries of this build are committed (traffic)
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh bench:cfg2 bench:cfg1 bench:cfg3 bench:cfg4 bench:cfg5 || exit $?
timeout -k 10 300 python -u bench.py --workload panda > gpurun_out/bench_panda.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload cfg2 --dtype f16x2 > gpurun_out/bench_cfg2_f16x2.log 2>&1
