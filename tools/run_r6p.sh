# round 6 (second session) closing run (a) on the final build: rocprofv3 kernel trace of the cfg2 line (+ its per-step
# timeline), FETCH/WRITE passes for cfg2 and cfg1, SQ counters of the headline kernel, U-Net roofline passes of
# cfg3 / cfg4 / cfg5 (their bench lines read these summaries as same-build traffic)
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh trace:cfg2 pmc:cfg2 pmc:cfg1 sqpmc:4096 || exit $?
python3 tools/step_timeline.py gpurun_out/prof/trace_cfg2 mlp_rw > gpurun_out/step_timeline_cfg2.txt 2>&1
bash tools/gpu.sh upmc:cfg3 upmc:cfg4 upmc:cfg5
