set -o pipefail
for v in nolastepi bar2; do bash tools/gpu.sh mlpab:$v || exit 1; done
for v in nolastepi bar2; do echo "== $v"; grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/mlpab_$v.log | tr '\n' ' '; echo; done
