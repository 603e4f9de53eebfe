#!/bin/bash
# A/B of sweep2 planner knobs (env, read once per process) on the latency-bound paths: the N=8
# rank of C4 (rank_sim: hoisted chain + one slice) and the C2 / C3 bench lines.  One fresh
# process per setting; results appended to gpurun_out/knobs.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/knobs.jsonl
for KV in "BASE=1" "TQ_SLICE_LANES=32" "TQ_S2D_BLOCKED=1" "TQ_S2D_NT=1" "TQ_S2_B4MIN=4096" "TQ_S2_B4MIN=2048" "TQ_S2_BLOCKS=0" "TQ_S2_EPI=0" "TQ_S2_MINLC=1"; do
  echo "== $KV"
  r=$(env $KV timeout -k 10 120 python3 scripts/rank_sim.py C4 2>/dev/null | tail -1) || exit 1
  echo "{\"knob\": \"$KV\", \"what\": \"C4 ranks\", \"res\": $r}" >> $OUT
  for C in C2 C3; do
    b=$(env $KV timeout -k 10 120 python3 bench.py --config $C --no-cpu-baseline --no-c5 --no-alt --no-other --steps 20 --warmup 5 2>/dev/null | tail -1) || exit 2
    echo "{\"knob\": \"$KV\", \"what\": \"$C\", \"ms\": $(echo $b | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')}" >> $OUT
  done
  tail -3 $OUT
done
