#!/bin/bash
# Round-2 GPU session 66: final bench line (roofline traffic from the batched-launch PMC summary)
# and the kernel trace of the same command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "b66 400 python bench.py" \
  "kt66 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt66 -o run -- python3 bench.py --no-cpu-baseline --no-c5 --no-alt"
