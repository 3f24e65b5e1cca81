set -o pipefail
timeout -k 10 300 python -u bench.py --workload cfg2 --no-cpu-baseline > gpurun_out/b_base.log 2>&1 || exit 1
MPCD_MLP_LAYOUT=rw32 timeout -k 10 300 python -u bench.py --workload cfg2 --no-cpu-baseline --no-shard-probe > gpurun_out/b_rw32.log 2>&1 || exit 1
MPCD_MLP_LAYOUT=rw32 MPCD_LIB=$PWD/mpc_via_diffusion_model_amd/libmpcd_rwunits.so timeout -k 10 300 python -u bench.py --workload cfg2 --no-cpu-baseline > gpurun_out/b_rwunits.log 2>&1 || exit 1
for lay in 32x8 rw32; do MPCD_MLP_LAYOUT=$lay MPCD_LIB=$PWD/mpc_via_diffusion_model_amd/libmpcd_prof.so DTYPE=f32x3 B=4096 timeout -k 10 300 python -u tools/layer_prof.py > gpurun_out/prof_$lay.txt 2>&1 || exit 1; done
