#!/bin/bash
# Round-2 GPU session 10: autograd (graph runtime), 2-rank native plan, full suite, bench (with C5 line).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "gputests 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread" \
  "bench 400 python bench.py --steps 10 --warmup 3"
