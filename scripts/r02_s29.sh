#!/bin/bash
# Round-2 GPU session 29: bench on the f16 split GEMM + rocprof kernel stats of the same command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "b29 300 python bench.py --no-cpu-baseline --no-c5" \
  "kt29 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt29 -o run -- python3 bench.py --no-cpu-baseline --no-c5 --no-alt"
