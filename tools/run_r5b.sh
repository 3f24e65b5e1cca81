# round 5: counters of the MLP samplers (two-term fp16 default, split-bf16 for the verdict's record) + traces + lines
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh sqpmc:4096 sqpmc:512 trace bench || exit $?
SQTAG=_x3 BENCH_ARGS="--dtype f32x3" bash tools/gpu.sh sqpmc:4096 sqpmc:512 || exit $?
cp -r gpurun_out/prof/trace_cfg2 gpurun_out/prof/trace_cfg2_h2
BENCH_ARGS="--dtype f32x3" bash tools/gpu.sh trace
