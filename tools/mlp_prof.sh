#!/bin/bash
# GPU box: per-layer cycle profile of the MLP sampler (experiment build libmpcd_prof.so, -DMPCD_PROF_LAYERS) at
# the headline batch and at the 512-candidate strong-scaling shard -> gpurun_out/mlp_prof_B<batch>.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for b in ${@:-4096 512}; do
  MPCD_LIB=$PWD/mpc_via_diffusion_model_amd/libmpcd_prof.so DTYPE=f32x3 B=$b timeout -k 10 300 \
    python -u tools/layer_prof.py > gpurun_out/mlp_prof_B$b.txt 2>&1 || exit $?
done
