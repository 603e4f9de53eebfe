#!/bin/bash
# A/B of library environment knobs on the C4 bench headline (one process per setting, same box).
# usage: [CFG=C3] scripts/ab_env.sh "label:VAR=v VAR2=v2" ... ("label:" alone = defaults)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for spec in "$@"; do
  label=${spec%%:*}
  envs=${spec#*:}
  echo "== $label ($envs)"
  env $envs timeout -k 10 200 python3 bench.py --config ${CFG:-C4} --no-cpu-baseline --no-c5 --no-alt --no-other --steps ${STEPS:-40} > gpurun_out/abe_$label.log 2>&1 || exit 1
  python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/abe_$label.log') if l.startswith('{')][-1])
r = d.get('roofline') or {}
print('$label', round(d['ms_per_step'], 4), 'ms/step', round(d['value'], 1), d['unit'], '| latency',
      (d.get('timing') or {}).get('latency_ms_per_step'), '| sweep avg us', r.get('avg_launch_us_events'),
      'GB/s', r.get('achieved'))"
done
