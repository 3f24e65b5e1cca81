cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m2 -E "gfx950|Marketing" > gpurun_out/rocminfo.txt
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-budget 8 > gpurun_out/bench.log 2>&1
