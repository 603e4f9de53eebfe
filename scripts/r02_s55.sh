#!/bin/bash
# Round-2 GPU session 55: slice lanes on C4 (TQ_LANE_ARENA_MB raised; 2 / 4 lanes of the 1.1-GiB
# per-slice working set) vs one lane: bench lines and C4 parity with lanes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "l1 300 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "l2 300 env TQ_LANE_ARENA_MB=4096 TQ_SLICE_LANES=2 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "l4 300 env TQ_LANE_ARENA_MB=8192 TQ_SLICE_LANES=4 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "l2t 300 env TQ_LANE_ARENA_MB=4096 TQ_SLICE_LANES=2 python -u -m pytest tests/test_fullsize_gpu.py -m gpu -x -q -rf --timeout 200 --timeout-method thread"
for f in l1 l2 l4; do grep '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value']/1e6,2), round(d['ms_per_step'],3), round(d['roofline']['avg_launch_ms'],3), d['hbm_kernels']['sweep_ms_per_step'])"; done
