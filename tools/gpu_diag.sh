# layer profiles of diagnostic builds listed in $DIAGS (libmpcd_<d>.so)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/diag
for v in $DIAGS; do
  MPCD_LIB=mpc_via_diffusion_model_amd/libmpcd_$v.so timeout -k 10 200 python tools/layer_prof.py > gpurun_out/diag/prof_$v.log 2>&1 || exit $?
done
