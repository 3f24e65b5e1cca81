# round 5 closing run on the committed build: GPU suite, smoke, every workload's line
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh tests smoke bench:cfg2 bench:cfg1 bench:cfg3 bench:cfg4 bench:cfg5 || exit $?
timeout -k 10 300 python -u bench.py --workload panda > gpurun_out/bench_panda.log 2>&1
