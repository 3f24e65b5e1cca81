# round 6: per-layer cycles per step of the final build against two timing experiments (wrong results): the weight
# stream removed (profnovm: zero-record descriptor) and the multi-pass layers' last epilogue dropped (profnle)
cd $GRAFT_REPO_ROOT
for v in prof profnovm profnle; do
  MPCD_LIB=$PWD/mpc_via_diffusion_model_amd/libmpcd_$v.so DTYPE=f32x3 B=4096 timeout -k 10 300 \
    python -u tools/layer_prof.py > gpurun_out/mlp_prof_$v.txt 2>&1 || exit $?
done
