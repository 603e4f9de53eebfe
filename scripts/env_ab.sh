#!/bin/bash
# A/B of HIP runtime environment settings on the latency-bound paths (fresh process each):
# C4 ranks (rank_sim), C2 and C3 bench lines.  Usage: scripts/env_ab.sh "A=1" "B=2 C=3" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/env_ab.jsonl
for KV in "$@"; do
  echo "== $KV"
  r=$(env $KV timeout -k 10 120 python3 scripts/rank_sim.py C4 2>/dev/null | tail -1) || exit 1
  echo "{\"env\": \"$KV\", \"what\": \"C4 ranks\", \"res\": $r}" >> $OUT
  for C in C2 C3; do
    b=$(env $KV timeout -k 10 120 python3 bench.py --config $C --no-cpu-baseline --no-c5 --no-alt --no-other --steps 20 --warmup 5 2>/dev/null | tail -1) || exit 2
    echo "{\"env\": \"$KV\", \"what\": \"$C\", \"ms\": $(echo $b | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')}" >> $OUT
  done
  tail -3 $OUT
done
