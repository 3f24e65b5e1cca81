set -o pipefail
cp mpc_via_diffusion_model_amd/libmpcd.so mpc_via_diffusion_model_amd/libmpcd_base.so
for v in base noslp base noslp; do bash tools/gpu.sh mlpab:$v || exit 1; grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/mlpab_$v.log | tr '\n' ' '; echo " <- $v"; done
