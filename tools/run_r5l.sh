# round 5: LDS bank-conflict counters of the fused U-Net programs (cfg5 fp16, cfg4 two-term fp16, cfg3 split bf16)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/uroof
export TMPDIR=/tmp
run() {  # $1 tag, rest: unet_perf args
  local tag=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA \
    -d gpurun_out/uroof/ldsc_$tag -o run -f csv -- python3 tools/unet_perf.py "$@" > gpurun_out/uroof/ldsc_$tag.log 2>&1
}
run cfg5 --B 131072 --H 64 --d 4 --C 12 --N 4 --schedule cosine --sampler ddpm_cfg --dtype f16 --reps 1 || exit $?
run cfg4h --B 65536 --H 64 --d 1 --C 5 --N 4 --schedule cosine --sampler ddpm_cfg --dtype f16x2 --reps 1 || exit $?
run cfg3 --B 16384 --H 32 --d 1 --C 2 --N 100 --steps 2 --dtype f32x3 --reps 1 || exit $?
