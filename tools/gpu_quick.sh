# quick loop: GPU tests, layer profile (prof build, if built), bench (f32x3 and f32)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; if [ $rc -gt 1 ]; then exit $rc; fi
if [ -f mpc_via_diffusion_model_amd/libmpcd_prof.so ]; then
  MPCD_LIB=mpc_via_diffusion_model_amd/libmpcd_prof.so DTYPE=f32x3 timeout -k 10 200 python tools/layer_prof.py > gpurun_out/layer_prof.log 2>&1 || exit $?
fi
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dtype f32x3 > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dtype f32 > gpurun_out/bench_f32.log 2>&1
