#!/bin/bash
# Round-2 GPU session 21: FP64 / complex128 LDS-DMA K-outer GEMM: parity, timing vs the generic
# kernel and torch, rocprof kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "g64t 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -rf -k gemm --timeout 120 --timeout-method thread" \
  "g64b 300 python scripts/gemm64_bench.py f64 c128" \
  "g64p 200 rocprofv3 --kernel-trace --stats -d gpurun_out/g64p -o run -- python3 scripts/gemm64_bench.py f64 c128 --layout=kouter"
