#!/bin/bash
# GPU box: U-Net roofline evidence for the BASELINE shapes. Per config: one kernel-trace pass and three
# PMC passes (FETCH_SIZE | WRITE_SIZE | MFMA busy + instruction counts), each its own rocprofv3 run over
# tools/unet_perf.py (a warm-up call that runs the tiling autotune, then one timed sample call). The
# trace pass writes its measured tilings to a tune cache that the PMC passes load, so all four passes run
# the same launches.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/uroof
declare -A ARGS=(
  [cfg3]="--B 16384 --H 32 --d 1 --C 2 --N 100 --dtype f32x3"
  [cfg5]="--B 131072 --H 64 --d 4 --C 12 --N 250 --schedule cosine --dtype f16"
  [cfg4]="--B 65536 --H 64 --d 1 --C 5 --N 100 --dtype f32x3"
)
for cfg in ${@:-cfg3 cfg5}; do
  a="${ARGS[$cfg]} --steps 1 --reps 1"
  export MPCD_UNET_TUNE_CACHE=gpurun_out/uroof/${cfg}_tune.txt
  rm -f $MPCD_UNET_TUNE_CACHE
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/uroof/${cfg}_trace -o run -f csv -- python3 tools/unet_perf.py $a > gpurun_out/uroof/${cfg}_trace.log 2>&1 || exit 1
  i=0
  for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"; do
    timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-include-regex "conv_mx|update_kernel|init_x" -d gpurun_out/uroof/${cfg}_p$i -o run -f csv -- python3 tools/unet_perf.py $a > gpurun_out/uroof/${cfg}_p$i.log 2>&1 || exit 1
    i=$((i+1))
  done
  echo "$cfg done"
done
