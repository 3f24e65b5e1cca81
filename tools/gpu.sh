#!/bin/bash
# The one GPU-box runner (start it through gpurun): tools/gpu.sh <job> [job ...], each job a word below,
# run in order; the first failing job ends the call (every GPU step has its own time limit).
#
#   tests[:<-k expr>]   pytest -m gpu (optionally -k <expr>)            -> gpurun_out/pytest_gpu.log
#   smoke               __graft_entry__.smoke()                          -> gpurun_out/smoke.log
#   bench[:<workload>]  bench.py --workload <workload> (default cfg2)     -> gpurun_out/bench_<workload>.log
#   trace[:<workload>]  rocprofv3 --kernel-trace --stats of that bench    -> gpurun_out/prof/trace_<workload>/
#   pmc[:<workload>]    FETCH_SIZE and WRITE_SIZE passes of that bench (one counter per pass, kernel trace
#                       only; tools/pmc_summary.py reads them)              -> gpurun_out/prof/pmc_<workload>_*/
#   upmc[:<cfg>]        U-Net per-launch roofline passes over tools/unet_perf.py (trace + FETCH_SIZE +
#                       WRITE_SIZE + MFMA busy), tune cache shared       -> gpurun_out/uroof/<cfg>_*
#   unet[:<cfg>]        tools/unet_perf.py timing of one sample call      -> gpurun_out/unet_<cfg>.log
#   mlpab:<variant>     cfg2 bench with libmpcd_<variant>.so (experiment build) -> gpurun_out/mlpab_<variant>.log
#   sqpmc[:<B>]        SQ instruction / wait / MFMA-busy counters of the cfg2 bench at B candidates (two passes)
#                                                                         -> gpurun_out/prof/sqpmc_<B>_*
#   l2pmc[:<workload>]  L1->L2 read requests and L2 hit / miss counters of that bench -> gpurun_out/prof/l2pmc_*
#
# Extra bench.py arguments for bench / trace / pmc come from $BENCH_ARGS; extra pytest arguments from
# $PYTEST_ARGS; extra unet_perf.py arguments from $UNET_ARGS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof gpurun_out/uroof

declare -A UARGS=(
  [cfg3]="--B 16384 --H 32 --d 1 --C 2 --N 100 --dtype f32x3"
  [cfg4]="--B 65536 --H 64 --d 1 --C 5 --N 100 --dtype f32x3"
  [cfg4h]="--B 65536 --H 64 --d 1 --C 5 --N 4 --schedule cosine --sampler ddpm_cfg --dtype f16x2"
  [cfg5]="--B 131072 --H 64 --d 4 --C 12 --N 250 --schedule cosine --dtype f16"
)

run_job() {
  local job=${1%%:*} arg=""
  [[ $1 == *:* ]] && arg=${1#*:}
  case $job in
    tests)
      local k=()
      [ -n "$arg" ] && k=(-k "$arg")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 240 --timeout-method thread \
        -p no:cacheprovider "${k[@]}" $PYTEST_ARGS > gpurun_out/pytest_gpu.log 2>&1
      local rc=$?
      echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
      return $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    bench)
      local w=${arg:-cfg2}
      timeout -k 10 600 python -u bench.py --workload "$w" $BENCH_ARGS > "gpurun_out/bench_$w.log" 2>&1 ;;
    trace)
      local w=${arg:-cfg2}
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof/trace_$w" -o run -f csv -- \
        python3 bench.py --workload "$w" --no-cpu-baseline --no-shard-probe $BENCH_ARGS > "gpurun_out/prof/trace_$w.log" 2>&1 ;;
    pmc)
      local w=${arg:-cfg2} c
      # the library the passes measure (tools/pmc_summary.py records it; bench.py compares it with the one it loads)
      sha256sum mpc_via_diffusion_model_amd/libmpcd.so | cut -d' ' -f1 > "gpurun_out/prof/pmc_${w}_lib.sha256"
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 300 rocprofv3 --pmc $c -d "gpurun_out/prof/pmc_${w}_$c" -o run -f csv -- \
          python3 bench.py --workload "$w" --no-cpu-baseline --steps 3 --warmup 1 $BENCH_ARGS \
          > "gpurun_out/prof/pmc_${w}_$c.log" 2>&1 || return $?
      done ;;
    mlpab)
      # cfg2 bench line of an experiment build (python -m mpc_via_diffusion_model_amd.build <variant> DEF=..)
      MPCD_LIB=$PWD/mpc_via_diffusion_model_amd/libmpcd_$arg.so timeout -k 10 300 python -u bench.py --workload cfg2 \
        --no-cpu-baseline $BENCH_ARGS > "gpurun_out/mlpab_$arg.log" 2>&1 ;;
    l2pmc)
      # cache counters of the cfg2 bench (one block per pass): L1 -> L2 read requests, L2 hits / misses
      local w=${arg:-cfg2} c i=0
      for c in "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TCC_HIT_sum TCC_MISS_sum"; do
        timeout -s KILL 120 rocprofv3 --pmc $c -d "gpurun_out/prof/l2pmc_${w}_$i" -o run -f csv -- \
          python3 bench.py --workload "$w" --no-cpu-baseline --no-shard-probe --steps 3 --warmup 1 $BENCH_ARGS \
          > "gpurun_out/prof/l2pmc_${w}_$i.log" 2>&1 || return $?
        i=$((i + 1))
      done ;;
    sqpmc)
      local b=${arg:-4096}${SQTAG} c i=0
      for c in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAVES" \
               "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
        timeout -s KILL 120 rocprofv3 --pmc $c -d "gpurun_out/prof/sqpmc_${b}_$i" -o run -f csv -- \
          python3 bench.py --workload cfg2 --candidates "${arg:-4096}" --no-cpu-baseline --no-shard-probe --steps 3 --warmup 1 $BENCH_ARGS \
          > "gpurun_out/prof/sqpmc_${b}_$i.log" 2>&1 || return $?
        i=$((i + 1))
      done ;;
    unet)
      local c=${arg:-cfg5}
      timeout -k 10 600 python -u tools/unet_perf.py ${UARGS[$c]} $UNET_ARGS > "gpurun_out/unet_$c.log" 2>&1 ;;
    upmc)
      # $UPMC_TAG: suffix of the output names (A/B of an environment switch, e.g. MPCD_FUSED_PERSIST=1)
      local c=${arg:-cfg5} i=0 ctr
      local a="${UARGS[$c]} --steps 1 --reps 1 $UNET_ARGS" n=${arg:-cfg5}$UPMC_TAG
      export MPCD_UNET_TUNE_CACHE=gpurun_out/uroof/${n}_tune.txt
      # the library the passes measure (tools/unet_roofline.py records it; bench.py compares it with the one it loads)
      sha256sum mpc_via_diffusion_model_amd/libmpcd.so | cut -d' ' -f1 > "gpurun_out/uroof/${n}_lib.sha256"
      rm -f "$MPCD_UNET_TUNE_CACHE"
      timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/uroof/${n}_trace" -o run -f csv -- \
        python3 tools/unet_perf.py $a > "gpurun_out/uroof/${n}_trace.log" 2>&1 || return $?
      for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"; do
        timeout -s KILL 300 rocprofv3 --pmc $ctr -d "gpurun_out/uroof/${n}_p$i" -o run -f csv -- \
          python3 tools/unet_perf.py $a > "gpurun_out/uroof/${n}_p$i.log" 2>&1 || return $?
        i=$((i + 1))
      done
      unset MPCD_UNET_TUNE_CACHE ;;
    *)
      echo "unknown job $1" >&2
      return 2 ;;
  esac
}

# refuse a library older than its sources (a snapshot taken before the rebuild finished)
for f in mpc_via_diffusion_model_amd/csrc/* include/mpcd.h; do
  if [ "$f" -nt mpc_via_diffusion_model_amd/libmpcd.so ]; then
    echo "[gpu.sh] STALE libmpcd.so: $f is newer; rebuild before the call" >&2
    exit 3
  fi
done
rocminfo 2>/dev/null | grep -m2 -E "gfx950|Marketing" > gpurun_out/rocminfo.txt
for j in "$@"; do
  echo "[gpu.sh] $j $(date +%T)"
  run_job "$j" || { rc=$?; echo "[gpu.sh] $j failed rc=$rc"; exit $rc; }
done
echo "[gpu.sh] done $(date +%T)"
