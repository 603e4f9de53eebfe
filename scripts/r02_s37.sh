#!/bin/bash
# Round-2 GPU session 37: f16 split GEMM with sched_group_barrier interleaving (TQ_GEMM_F16_VAR:
# 0 = 4 waves of 64x64 interleaved, 1 = 8 waves of 64x32 interleaved, 2 / 3 = the same without).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "k37 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -rf -k gemm_c64 --timeout 120 --timeout-method thread" \
  "k37b 300 env TQ_GEMM_F16_VAR=1 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -rf -k 'gemm_c64 and f16' --timeout 120 --timeout-method thread" \
  "v0 100 env TQ_GEMM_F16_VAR=0 python scripts/gemm_c64_bench.py --bench-shape" \
  "v1 100 env TQ_GEMM_F16_VAR=1 python scripts/gemm_c64_bench.py --bench-shape" \
  "v2 100 env TQ_GEMM_F16_VAR=2 python scripts/gemm_c64_bench.py --bench-shape" \
  "v3 100 env TQ_GEMM_F16_VAR=3 python scripts/gemm_c64_bench.py --bench-shape"
