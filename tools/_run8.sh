set -o pipefail
export MPCD_SPREAD_LOG=$PWD/gpurun_out/spread_ratios.tsv
rm -f $MPCD_SPREAD_LOG
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
for lay in 16x8 rw16; do MPCD_MLP_LAYOUT=$lay timeout -k 10 300 python -u bench.py --workload cfg1 --no-cpu-baseline > gpurun_out/b_cfg1_$lay.log 2>&1 || exit 1; done
