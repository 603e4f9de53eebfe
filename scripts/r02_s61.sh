#!/bin/bash
# Round-2 GPU session 61: pre-split operands with the lane-batched GEMM (one window flag per
# batch): presplit parity tests, then same-box A/B of the C4 bench, default vs TQ_GEMM_PRESPLIT=1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "p61 300 python -u -m pytest tests/test_presplit_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q -rf --timeout 200 --timeout-method thread" \
  "d0a 300 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "d1a 300 env TQ_GEMM_PRESPLIT=1 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "d0b 300 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "d1b 300 env TQ_GEMM_PRESPLIT=1 python bench.py --no-cpu-baseline --no-c5 --no-alt"
for f in d0a d1a d0b d1b; do grep '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value']/1e6,2), round(d['ms_per_step'],3), round(d['roofline']['avg_launch_ms'],3), round(d['hbm_kernels']['sweep_ms_per_step'],3))"; done
