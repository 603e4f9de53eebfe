#!/bin/bash
# Round-2 GPU session 50: HEAD after the sweep2 epilogue (pre-split GEMM opt-in): full GPU suite,
# smoke, full bench (CPU baseline, alt kernels, C5 line), kernel trace of the bench command,
# C3 / C2 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "t50 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread" \
  "s50 200 python -c 'import __graft_entry__ as g; g.smoke()'" \
  "b50 400 python bench.py" \
  "kt50 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt50 -o run -- python3 bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "c3_50 300 python bench.py --config C3" \
  "c2_50 300 python bench.py --config C2"
