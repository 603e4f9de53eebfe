#!/bin/bash
# Round-2 GPU session 30: producer-fused operand max (sweep2 -> f16-split GEMM): full GPU suite,
# smoke, bench, f16 GEMM PMC passes + kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "t30 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread" \
  "s30 200 python -c 'import __graft_entry__ as g; g.smoke()'" \
  "b30 400 python bench.py" \
  "p30 500 bash scripts/pmc_gemm_f16.sh"
