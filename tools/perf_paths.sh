cd $GRAFT_REPO_ROOT
bash tools/gpu.sh "tests:fused_philox or uncovered" || exit $?
for c in cfg5 cfg3 cfg4; do
  for p in fused layered; do
    UNET_ARGS="--path $p --steps 10 --reps 2" bash tools/gpu.sh unet:$c || exit $?
    cp gpurun_out/unet_$c.log gpurun_out/perf_${c}_$p.log
  done
done
