cd /root/repo
export TMPDIR=/tmp
for v in default nofence nofence_noslp; do
  if [ $v = default ]; then L=""; else L="$PWD/mpc_via_diffusion_model_amd/libmpcd_$v.so"; fi
  MPCD_LIB=$L MPCD_UNET_FUSED=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_unet_bench_sizes.py -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/hz_$v.log 2>&1
  echo "$v rc=$?" >> gpurun_out/hz_summary.txt
done
