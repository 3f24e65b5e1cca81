set -o pipefail
bash tools/gpu.sh upmc:cfg3 || exit 1
UPMC_TAG=_pers MPCD_FUSED_PERSIST=1 bash tools/gpu.sh upmc:cfg3 || exit 1
bash tools/gpu.sh upmc:cfg4 || exit 1
UPMC_TAG=_pers MPCD_FUSED_PERSIST=1 bash tools/gpu.sh upmc:cfg4 || exit 1
ls gpurun_out/uroof
