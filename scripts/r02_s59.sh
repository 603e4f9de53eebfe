#!/bin/bash
# Round-2 GPU session 59 (round-end state): full GPU suite, smoke, full bench and the rocprof
# kernel trace of the same bench command, single-GPU rank projection.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "t59 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread" \
  "s59 200 python -c 'import __graft_entry__ as g; g.smoke()'" \
  "b59 400 python bench.py" \
  "kt59 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt59 -o run -- python3 bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "r59 200 python scripts/rank_sim.py C4"
