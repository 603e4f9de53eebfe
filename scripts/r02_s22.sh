#!/bin/bash
# Round-2 GPU session 22 (re-entry check): full GPU suite, smoke, default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "t22 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread" \
  "s22 200 python -c 'import __graft_entry__ as g; g.smoke()'" \
  "b22 400 python bench.py"
