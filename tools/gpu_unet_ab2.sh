# Same-box A/B/A/B of two libmpcd builds on the cfg5-shape forward (fresh autotune per process)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/unet_ab2.log
: > $L
for rep in 1 2; do
for lib in libmpcd.so $ALTS; do
  echo "$lib" >> $L
  MPCD_LIB=mpc_via_diffusion_model_amd/$lib timeout -k 10 200 python tools/unet_perf.py --B ${B:-131072} --H 64 --d ${D:-4} --C ${C:-12} --steps 3 --reps 1 --dtype ${DT:-f16} --schedule cosine --N 250 >> $L 2>&1 || exit $?
done
done
