# round 5 final evidence, part 1: the whole GPU suite, smoke, the cfg2 headline line (+ CPU baseline), its kernel
# trace, FETCH/WRITE and SQ passes of the fp16 MLP kernel
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh tests smoke bench:cfg2 trace:cfg2 pmc:cfg2 || exit $?
SQTAG=_h2 bash tools/gpu.sh sqpmc:4096 sqpmc:512
