# round 5: the fp16 MLP kernel with swizzled activation rows - parity, cfg2 line, SQ LDS counters, layer profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp_h2.py tests/test_gpu_headline.py tests/test_gpu_mlp.py tests/test_gpu_rollout.py -x -q --timeout 300 --timeout-method thread > gpurun_out/mlp_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_h2.log 2>&1 || exit $?
true
MPCD_LIB=$PWD/mpc_via_diffusion_model_amd/libmpcd_prof.so DTYPE=f16x2 H2=1 B=4096 timeout -k 10 300 \
  python -u tools/layer_prof.py > gpurun_out/h2_prof_B4096.txt 2>&1
