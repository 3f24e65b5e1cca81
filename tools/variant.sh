#!/bin/bash
# Experiment build that differs from the product only in one source: tools/variant.sh <name> <source.hip> DEF=.. ...
# (the product's other objects are copied in and kept, so only <source> is recompiled with the defines)
cd "$(dirname "$0")/.." || exit 1
v=$1; src=$2; shift 2
mkdir -p mpc_via_diffusion_model_amd/_build_$v
cp -p mpc_via_diffusion_model_amd/_build/*.o mpc_via_diffusion_model_amd/_build_$v/
touch mpc_via_diffusion_model_amd/_build_$v/*.o
rm -f mpc_via_diffusion_model_amd/_build_$v/${src%.hip}.o
python -m mpc_via_diffusion_model_amd.build $v "$@"
