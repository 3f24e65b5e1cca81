# round 6: the U-Net workloads' lines again, now that their PMC summaries of this build are committed (traffic
# same_build)
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh bench:cfg3 bench:cfg4 bench:cfg5
