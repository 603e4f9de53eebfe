#!/bin/bash
# Round-2 GPU session 42: bench lines for the other amplitude configs (C3: 40q d16, 64 slices;
# C2: 30q d14, one amplitude) with their CPU baselines; C3 kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "c3 400 python bench.py --config C3 --no-c5 --no-alt" \
  "c2 400 python bench.py --config C2 --no-c5 --no-alt" \
  "kc3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kc3 -o run -- python3 bench.py --config C3 --no-cpu-baseline --no-c5 --no-alt"
