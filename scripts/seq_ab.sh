#!/bin/bash
# A/B of the chain-launch knobs on C2 / C3 (bench lines) and C4 ranks: each setting in a fresh
# process, interleaved twice.  Usage: scripts/seq_ab.sh "TQ_S2_SEQ=1" "TQ_S2_SEQ=0" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/seq_ab.jsonl
for rep in 1 2; do
  for KV in "$@"; do
    r=$(env $KV timeout -k 10 150 python3 scripts/rank_sim.py C4 2>/dev/null | tail -1) || exit 3
    echo "{\"env\": \"$KV\", \"what\": \"C4 N8 rank\", \"ms\": $(echo $r | python3 -c 'import json,sys; print(json.load(sys.stdin)["rank_ms_N8"])')}" | tee -a $OUT
    for C in C2 C3; do
      b=$(env $KV timeout -k 10 120 python3 bench.py --config $C --no-cpu-baseline --no-c5 --no-alt --no-other --steps 50 --warmup 10 2>/dev/null | tail -1) || exit 2
      echo "{\"env\": \"$KV\", \"what\": \"$C\", \"ms\": $(echo $b | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')}" | tee -a $OUT
    done
  done
done
