# A/B the MLP sampler variants listed in $VARIANTS (libmpcd_<v>.so + libmpcd_<v>prof.so): bench + layer profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for v in $VARIANTS; do
  MPCD_LIB=mpc_via_diffusion_model_amd/libmpcd_$v.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab/bench_$v.log 2>&1 || exit $?
  if [ -f mpc_via_diffusion_model_amd/libmpcd_${v}prof.so ]; then
    MPCD_LIB=mpc_via_diffusion_model_amd/libmpcd_${v}prof.so timeout -k 10 200 python tools/layer_prof.py > gpurun_out/ab/prof_$v.log 2>&1 || exit $?
  fi
done
