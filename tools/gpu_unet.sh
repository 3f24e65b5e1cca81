cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_unet.py -x -q -p no:cacheprovider > gpurun_out/pytest_unet.log 2>&1
echo "rc=$?" >> gpurun_out/pytest_unet.log
