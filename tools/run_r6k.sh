# round 6: U-Net roofline passes (trace, FETCH_SIZE, WRITE_SIZE, MFMA busy + SQ instruction counts) of cfg3, cfg4
# (f32x3, the bench default since round 6) and cfg5 (f16) on the final build
cd $GRAFT_REPO_ROOT
bash tools/gpu.sh upmc:cfg3 upmc:cfg4 upmc:cfg5
