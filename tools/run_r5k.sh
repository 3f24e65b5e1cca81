# round 5 final evidence, part 2: the other workloads' lines on the final build and the cfg4 fp16x2 roofline passes
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh bench:cfg1 bench:cfg3 bench:cfg4 bench:cfg5 upmc:cfg4h || exit $?
timeout -k 10 300 python -u bench.py --workload panda > gpurun_out/bench_panda.log 2>&1
