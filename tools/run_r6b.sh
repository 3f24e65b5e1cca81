# round 6: the f32x3 cfg2 line (swizzle, fenced split, log2(e) fold), GPU suite, SQ counters, per-layer profile
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh bench:cfg2 tests sqpmc:4096 || exit $?
bash tools/mlp_prof.sh 4096 512
