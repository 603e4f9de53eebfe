#!/bin/bash
# Round-2 GPU session 60: f16 split GEMM on a 4-slot LDS ring (one barrier per two K-steps,
# gemm_f16_var 3): kernel parity on every variant, then C4 bench default vs ring, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "k60 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -rf --timeout 200 --timeout-method thread" \
  "v0a 300 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "v3a 300 env TQ_GEMM_F16_VAR=3 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "v0b 300 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "v3b 300 env TQ_GEMM_F16_VAR=3 python bench.py --no-cpu-baseline --no-c5 --no-alt"
for f in v0a v3a v0b v3b; do grep '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value']/1e6,2), round(d['ms_per_step'],3), round(d['roofline']['avg_launch_ms'],3))"; done
