cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_unet
timeout -k 10 300 python tools/unet_perf.py --B 16384 --H 32 --C 2 --steps 10 > gpurun_out/unet_perf.log 2>&1 || exit $?
timeout -k 10 300 python tools/unet_perf.py --B 8192 --H 64 --C 5 --steps 5 >> gpurun_out/unet_perf.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_unet -o run -f csv -- python3 tools/unet_perf.py --B 16384 --H 32 --C 2 --steps 4 --reps 1 > gpurun_out/prof_unet/log 2>&1
