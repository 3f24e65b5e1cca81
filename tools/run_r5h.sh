# round 5: per-layer profile of the fp16 MLP kernel after the conflict-free strides; then the U-Net f16x2 checks
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 4096 512; do
  MPCD_LIB=$PWD/mpc_via_diffusion_model_amd/libmpcd_prof.so DTYPE=f16x2 H2=1 B=$b timeout -k 10 300 \
    python -u tools/layer_prof.py > gpurun_out/h2_prof_B$b.txt 2>&1 || exit $?
done
bash tools/run_r5f.sh
