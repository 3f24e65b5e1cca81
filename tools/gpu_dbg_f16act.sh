timeout -k 10 200 python tools/debug_f16act.py > gpurun_out/dbg_f16act.log 2>&1 && bash tools/gpu_f16act.sh
