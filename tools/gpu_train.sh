# Training-step parity (tests/test_gpu_train.py) and throughput (tools/train_bench.py) on one GPU.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_train.log 2>&1 || exit $?
for cfg in "--net mlp --B 4096" "--net unet --B 256" "--net unet --B 1024"; do
  timeout -k 10 120 python tools/train_bench.py $cfg >> gpurun_out/train_bench.txt 2>&1 || exit $?
done
