#!/bin/bash
# Round-2 GPU session 38: settled f16 GEMM (8 waves, interleaved): full GPU suite, smoke, bench,
# f16 GEMM PMC passes + kernel trace of the bench command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "t38 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread" \
  "s38 200 python -c 'import __graft_entry__ as g; g.smoke()'" \
  "b38 400 python bench.py" \
  "p38 500 bash scripts/pmc_gemm_f16.sh"
