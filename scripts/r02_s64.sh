#!/bin/bash
# Round-2 GPU session 64: C4 with 4 lanes, f16 GEMM tile variants on the batched launch
# (default 8 waves of 64x32 vs 4 waves of 64x64), alternating on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "w0a 300 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "w1a 300 env TQ_GEMM_F16_VAR=1 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "w0b 300 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "w1b 300 env TQ_GEMM_F16_VAR=1 python bench.py --no-cpu-baseline --no-c5 --no-alt"
for f in w0a w1a w0b w1b; do grep '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value']/1e6,2), round(d['ms_per_step'],3), round(d['roofline']['avg_launch_ms'],3))"; done
