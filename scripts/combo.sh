#!/bin/bash
# Combined planner settings (each a fresh process) on C4 ranks, C2, C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/combo.jsonl
for KV in "BASE=1" "TQ_SLICE_LANES=32 TQ_S2_MINLC=1" "TQ_SLICE_LANES=32 TQ_S2_MINLC=1 TQ_S2_B4MIN=4096" "TQ_SLICE_LANES=32 TQ_S2_B4MIN=4096"; do
  echo "== $KV"
  r=$(env $KV timeout -k 10 120 python3 scripts/rank_sim.py C4 2>/dev/null | tail -1) || exit 1
  echo "{\"knob\": \"$KV\", \"what\": \"C4 ranks\", \"res\": $r}" >> $OUT
  for C in C2 C3; do
    b=$(env $KV timeout -k 10 120 python3 bench.py --config $C --no-cpu-baseline --no-c5 --no-alt --no-other --steps 20 --warmup 5 2>/dev/null | tail -1) || exit 2
    echo "{\"knob\": \"$KV\", \"what\": \"$C\", \"ms\": $(echo $b | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')}" >> $OUT
  done
  tail -3 $OUT
done
