# round 6, first call: GPU suite on the swizzled split-bf16 MLP kernel, the f32x3 cfg2 line, its SQ counters
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh tests bench:cfg2 sqpmc:4096
