#!/bin/bash
# A/B of the cooperative chain launch on C2 (bench lines), each setting in a fresh process,
# interleaved three times.  Usage: scripts/coop_ab.sh "TQ_S2_COOP=1" "TQ_S2_COOP=0" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/coop_ab.jsonl
for rep in 1 2 3; do
  for KV in "$@"; do
    b=$(env $KV timeout -k 10 120 python3 bench.py --config C2 --no-cpu-baseline --no-c5 --no-alt --no-other --steps 200 --warmup 20 2>/dev/null | tail -1) || exit 2
    echo "{\"env\": \"$KV\", \"what\": \"C2\", \"ms\": $(echo $b | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')}" | tee -a $OUT
  done
done
