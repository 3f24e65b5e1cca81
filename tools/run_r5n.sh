# round 5 final evidence (after the MLP row swizzle and the host-path changes): GPU suite, smoke, cfg2 / cfg1 lines,
# cfg2 kernel trace, FETCH/WRITE and SQ passes
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh tests smoke bench:cfg2 trace:cfg2 pmc:cfg2 bench:cfg1 || exit $?
SQTAG=_final bash tools/gpu.sh sqpmc:4096 sqpmc:512
