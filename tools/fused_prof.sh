#!/bin/bash
# GPU box: per-op timing of the fused U-Net kernel (MPCD_FUSED_PROF) at the cfg5 / cfg3 / cfg4 shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for c in ${@:-cfg5 cfg3}; do
  case $c in
    cfg3) a="--B 16384 --H 32 --d 1 --C 2 --N 100 --dtype f32x3" ;;
    cfg4) a="--B 65536 --H 64 --d 1 --C 5 --N 100 --dtype f32x3" ;;
    cfg5) a="--B 131072 --H 64 --d 4 --C 12 --N 250 --schedule cosine --dtype f16" ;;
  esac
  MPCD_FUSED_PROF=gpurun_out/fprof_$c.bin timeout -k 10 300 python -u tools/unet_perf.py $a --path fused --steps 3 --reps 1 \
    > gpurun_out/fprof_$c.log 2>&1 || exit $?
  python tools/fused_prof.py gpurun_out/fprof_$c.bin > gpurun_out/fprof_$c.txt || exit $?
done
