#!/bin/bash
# Round-2 GPU session 6 (instrumented build): sweep2 phase timing of one C4 execute.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh "s2t 200 python scripts/sweep_timing.py C4"
