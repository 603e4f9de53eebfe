#!/bin/bash
# Round-2 GPU session 58: C4 with 8 slice lanes (budget raised) vs the default 4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "m4 300 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "m8 300 env TQ_LANE_ARENA_MB=12288 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "m4b 300 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "m8b 300 env TQ_LANE_ARENA_MB=12288 python bench.py --no-cpu-baseline --no-c5 --no-alt"
for f in m4 m8 m4b m8b; do grep '^{' gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value']/1e6,2), round(d['ms_per_step'],3), round(d['roofline']['avg_launch_ms'],3), round(d['hbm_kernels']['sweep_ms_per_step'],3), d['plan']['arena_GiB'])"; done
