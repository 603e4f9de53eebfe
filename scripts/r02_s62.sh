#!/bin/bash
# Round-2 GPU session 62: round-end check after the pre-split/lanes change: full GPU suite + smoke.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "t62 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread" \
  "s62 200 python -c 'import __graft_entry__ as g; g.smoke()'"
