#!/bin/bash
# Round-2 GPU session 57: full bench after the lane-aware profiling counts; C5 line in a child process.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "b57 400 python bench.py" \
  "c3_57 300 python bench.py --config C3 --no-c5 --no-alt"
