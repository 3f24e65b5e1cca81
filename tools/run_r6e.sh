# round 6: counter-synchronised split-bf16 MLP variants (f1: signal wait, no sleep; f2: no signal wait; f3: f2 without
# carries) against the barrier product; bit-identity tests on the variants without the signal wait
cd $GRAFT_REPO_ROOT
export BENCH_ARGS="--no-shard-probe"
bash tools/gpu.sh "tests:mlp or headline" bench:cfg2 mlpab:f1 mlpab:f2 mlpab:f3 || exit $?
for v in f2 f3; do
  MPCD_LIB=$PWD/mpc_via_diffusion_model_amd/libmpcd_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py \
    tests/test_gpu_headline.py -x -q --timeout 120 --timeout-method thread -k "f32x3 or layout" > gpurun_out/${v}_tests.log 2>&1 || exit $?
done
