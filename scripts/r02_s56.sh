#!/bin/bash
# Round-2 GPU session 56: HEAD with slice lanes (C3: 8, C4: 4 within the 6-GiB budget) and C5
# candidates on streams: full GPU suite, smoke, full bench, kernel trace, C3 / C2 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "t56 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread" \
  "s56 200 python -c 'import __graft_entry__ as g; g.smoke()'" \
  "b56 400 python bench.py" \
  "kt56 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt56 -o run -- python3 bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "c3_56 300 python bench.py --config C3 --no-c5 --no-alt" \
  "c2_56 300 python bench.py --config C2 --no-c5 --no-alt"
