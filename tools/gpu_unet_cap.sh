# U-Net LDS-cap experiment (occupancy vs rows per workgroup), cfg3 shape.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/unet_cap.log
: > $L
for cap in 163840 81920 53248 40960; do
  for dt in f16 f32x3; do
    echo "cap=$cap" >> $L
    MPCD_UNET_LDS_CAP=$cap timeout -k 10 200 python tools/unet_perf.py --B 16384 --H 32 --d 1 --C 2 --steps 4 --reps 1 --dtype $dt >> $L 2>&1 || exit $?
  done
done
