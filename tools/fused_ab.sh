#!/bin/bash
# GPU box: fused U-Net configuration A/B at the BASELINE shapes (tools/unet_perf.py ms per CFG evaluation):
# tools/fused_ab.sh "<ROWS>:<WAVES>" ...   (empty pair = the default configuration) -> gpurun_out/fab_*.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
for rw in "$@"; do
  r=${rw%%:*}; w=${rw##*:}
  for c in cfg5 cfg3; do
    case $c in
      cfg3) a="--B 16384 --H 32 --d 1 --C 2 --N 100 --dtype f32x3" ;;
      cfg5) a="--B 131072 --H 64 --d 4 --C 12 --N 250 --schedule cosine --dtype f16" ;;
    esac
    MPCD_FUSED_ROWS=$r MPCD_FUSED_WAVES=$w timeout -k 10 300 python -u tools/unet_perf.py $a --path fused \
      > gpurun_out/fab_${c}_R${r}W${w}.log 2>&1
    echo "$c R=$r W=$w: $(grep -h 'ms/eval' gpurun_out/fab_${c}_R${r}W${w}.log | tail -1 | sed 's/.*-> //')" >> gpurun_out/fab_summary.txt
  done
done
