# PMC passes over the U-Net conv kernels (cfg3 shape, one CFG evaluation after a warm-up), one pass per
# counter group, kernel-trace only.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/upmc
run() { timeout -s KILL 120 rocprofv3 --pmc $3 --kernel-include-regex conv_mx -d gpurun_out/upmc/$1_$2 -o run -f csv -- python3 tools/unet_perf.py --B 16384 --H 32 --C 2 --steps 1 --reps 1 --dtype $1 > gpurun_out/upmc/$1_$2.log 2>&1; }
for dt in f16 f32x3; do
  run $dt a "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" || exit $?
  run $dt b "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES" || exit $?
  run $dt c "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MFMA" || exit $?
  run $dt d "FETCH_SIZE" || exit $?
  run $dt e "WRITE_SIZE" || exit $?
done
