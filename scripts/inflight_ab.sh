#!/bin/bash
# A/B of library environment knobs on C4 blocks per second with 1 and 2 blocks in flight
# (probes/inflight.py; one process per setting, same box).
# usage: scripts/inflight_ab.sh "label:VAR=v VAR2=v2" ... ("label:" alone = defaults)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for spec in "$@"; do
  label=${spec%%:*}; envs=${spec#*:}
  r=$(env $envs timeout -k 10 120 python3 probes/inflight.py C4 1 2 2>/dev/null | grep inflight | tr '\n' ' ') || exit 1
  echo "$label $r"
done
