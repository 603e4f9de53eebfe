#!/bin/bash
# A/B of complex64 boundary-GEMM variants on the C4 bench: headline per variant, then one PMC pass
# per variant (clock, MFMA busy) over the split kernel.  usage: scripts/ab_gemm.sh VAR [VAR ...]
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
B="python3 bench.py --no-cpu-baseline --no-c5 --no-alt --no-other"
for v in "$@"; do
  echo "== bench var $v"
  TQ_GEMM_F16_VAR=$v timeout -k 10 200 $B --steps 20 > gpurun_out/ab_b$v.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_b$v.log') if l.startswith('{')][-1]); r=d['roofline']; print('var $v', round(d['ms_per_step'],3), 'ms/step', round(r['avg_launch_ms'],3), 'ms/GEMM', round(d['value']/1e6,2), 'M amp/s')"
done
for v in "$@"; do
  echo "== pmc var $v"
  TQ_GEMM_F16_VAR=$v timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    --kernel-include-regex split_kernel --output-format csv -d gpurun_out/ab$v/pmc -o run -- $B --steps 2 --warmup 1 > gpurun_out/ab_p$v.log 2>&1 || exit 2
  python3 scripts/pmc_summary.py split_kernel gpurun_out/ab$v | head -12
done
