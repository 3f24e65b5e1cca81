# Workgroup duration vs co-resident workgroups per CU (LDS padding) for two cfg5 convs, tuned tilings kept
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/occ
cp profiles/r2_unet_tune_cfg5.txt /tmp/tune5.txt
for pad in 0 20000 45000 90000; do
  for L in 14 2; do
    MPCD_UNET_LDS_PAD=$pad MPCD_UNET_WGTRACE=$L MPCD_UNET_TUNE_CACHE=/tmp/tune5.txt timeout -k 10 120 python tools/unet_perf.py --B 131072 --H 64 --d 4 --C 12 --steps 1 --reps 1 --dtype f16 --schedule cosine --N 250 --fuse 0 > gpurun_out/occ/p${pad}_L$L.log 2>&1 || exit 1
    mv gpurun_out/wgtrace_L$L.bin gpurun_out/occ/wgtrace_p${pad}_L$L.bin
  done
done
