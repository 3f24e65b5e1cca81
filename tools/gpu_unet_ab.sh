# A/B of libmpcd builds on the cfg5-shape forward (fresh autotune per build: no tune cache)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/unet_ab.log
: > $L
for lib in libmpcd.so $ALTS; do
  echo "$lib" >> $L
  MPCD_LIB=mpc_via_diffusion_model_amd/$lib timeout -k 10 200 python tools/unet_perf.py --B ${B:-131072} --H 64 --d ${D:-4} --C ${C:-12} --steps 3 --reps 2 --dtype ${DT:-f16} --schedule cosine --N 250 >> $L 2>&1 || exit $?
done
