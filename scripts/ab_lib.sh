#!/bin/bash
# A/B of library builds (e.g. a diagnostic build under scratch/) on the C4 bench: headline per
# build, then one PMC pass per build (clock, MFMA busy) over the split GEMM kernel.
# usage: scripts/ab_lib.sh "label:" "label2:scratch/libdiag.so" ...  ("label:" = lib/libtneqhip.so)
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
B="python3 bench.py --no-cpu-baseline --no-c5 --no-alt --no-other"
libenv() { [ -n "$1" ] && echo "TNEQHIP_LIB=$PWD/$1"; }
for spec in "$@"; do
  l=${spec%%:*}; p=${spec#*:}
  echo "== bench $l"
  env $(libenv "$p") timeout -k 10 200 $B --steps 20 > gpurun_out/abl_b$l.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/abl_b$l.log') if l.startswith('{')][-1]); r=d['roofline']; print('$l', round(d['ms_per_step'],3), 'ms/step', round(r['avg_launch_ms'],3), 'ms/GEMM', round(d['value']/1e6,2), 'M amp/s')"
done
for spec in "$@"; do
  l=${spec%%:*}; p=${spec#*:}
  echo "== pmc $l"
  env $(libenv "$p") timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    --kernel-include-regex split_kernel --output-format csv -d gpurun_out/abl$l/pmc -o run -- $B --steps 2 --warmup 1 > gpurun_out/abl_p$l.log 2>&1 || exit 2
  python3 scripts/pmc_summary.py split_kernel gpurun_out/abl$l | head -12
done
