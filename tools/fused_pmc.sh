#!/bin/bash
# GPU box: PMC passes (one counter block set per pass, kernel trace only) over the fused U-Net kernel at a
# BASELINE shape: tools/fused_pmc.sh cfg5|cfg3|cfg4 [path]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
c=${1:-cfg5}; path=${2:-fused}
case $c in
  cfg3) a="--B 16384 --H 32 --d 1 --C 2 --N 100 --dtype f32x3" ;;
  cfg4) a="--B 65536 --H 64 --d 1 --C 5 --N 100 --dtype f32x3" ;;
  cfg5) a="--B 131072 --H 64 --d 4 --C 12 --N 250 --schedule cosine --dtype f16" ;;
esac
mkdir -p gpurun_out/fpmc
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM_RD" "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-include-regex "unet_fused|conv_mx" -d gpurun_out/fpmc/${c}_${path}_p$i -o run -f csv -- \
    python3 tools/unet_perf.py $a --path $path --steps 2 --reps 1 > gpurun_out/fpmc/${c}_${path}_p$i.log 2>&1 || exit $?
  i=$((i + 1))
done
