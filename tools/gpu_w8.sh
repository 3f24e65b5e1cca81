# A/B the 8-wave split-bf16 MLP kernel (libmpcd_w8.so) against the product build: MLP parity, then bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
MPCD_LIB=mpc_via_diffusion_model_amd/libmpcd_w8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/pytest_w8.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/ab/bench_w4_$i.log 2>&1 || exit $?
  MPCD_LIB=mpc_via_diffusion_model_amd/libmpcd_w8.so timeout -k 10 200 python bench.py --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/ab/bench_w8_$i.log 2>&1 || exit $?
done
