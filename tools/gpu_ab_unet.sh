# A/B the U-Net sampler: product library vs libmpcd_prev.so (previous commit), interleaved, same box
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/ab_unet.log
: > $L
for dt in f32x3 f16; do
  for lib in prev cur prev cur; do
    if [ $lib = prev ]; then export MPCD_LIB=mpc_via_diffusion_model_amd/libmpcd_prev.so; else unset MPCD_LIB; fi
    echo "lib=$lib" >> $L
    timeout -k 10 200 python tools/unet_perf.py --B 16384 --H 32 --d 1 --C 2 --steps 10 --reps 1 --dtype $dt >> $L 2>&1 || exit $?
  done
done
