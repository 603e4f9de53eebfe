#!/bin/bash
# Headline (C4 bitstring blocks) against the HIP hardware-queue count and the blocks in flight,
# one process per setting on the same box.
# usage: scripts/hwq_sweep.sh "queues:inflight[:group]" ...   (e.g. "4:4" "8:4" "8:6" "8:8")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for spec in "$@"; do
  IFS=: read -r q i g <<< "$spec"
  g=${g:-1}
  label="q${q}_i${i}_g${g}"
  echo "== $label"
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 bench.py --config ${CFG:-C4} --no-cpu-baseline --no-c5 --no-alt \
    --no-other --steps ${STEPS:-40} --inflight "$i" --group "$g" > gpurun_out/hwq_$label.log 2>&1 || exit 1
  python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/hwq_$label.log') if l.startswith('{')][-1])
r = d.get('roofline') or {}
print('$label', round(d['ms_per_step'], 4), 'ms/step', round(d['value'] / 1e9, 3), 'G', d['unit'], '| latency',
      (d.get('timing') or {}).get('latency_ms_per_step'), '| sweep avg us', r.get('avg_launch_us_events'))"
done
