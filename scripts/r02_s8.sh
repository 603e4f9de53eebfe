#!/bin/bash
# Round-2 GPU session 8: full GPU suite + smoke + bench after SGDG kernel / sweep2 pipeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "gputests 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread" \
  "smoke 200 python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench 300 python bench.py --steps 10 --warmup 3" \
  "ranksim 300 python scripts/rank_sim.py C4"
