set -o pipefail
for v in prof profnd; do
  MPCD_LIB=$PWD/mpc_via_diffusion_model_amd/libmpcd_$v.so DTYPE=f32x3 timeout -k 10 300 python -u tools/layer_prof.py > gpurun_out/layer_$v.log 2>&1 || exit 1
done
paste gpurun_out/layer_prof.log gpurun_out/layer_profnd.log
