# round 6: split-bf16 MLP tuning variants (pf3: operand fragments 3 k-chunks ahead; te: next step's cond tables
# written after Linear 11; pf3te: both) against the product; MLP parity on the product and on te
cd $GRAFT_REPO_ROOT
export BENCH_ARGS="--no-shard-probe"
bash tools/gpu.sh "tests:mlp or headline" bench:cfg2 mlpab:pf3 mlpab:te mlpab:pf3te || exit $?
MPCD_LIB=$PWD/mpc_via_diffusion_model_amd/libmpcd_te.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py \
  tests/test_gpu_headline.py -x -q --timeout 120 --timeout-method thread -k "f32x3 or layout" > gpurun_out/te_tests.log 2>&1
