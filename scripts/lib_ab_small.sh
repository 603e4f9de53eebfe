#!/bin/bash
# A/B of two library builds on the latency-bound lines: C2 / C3 bench lines and the C4 N = 8 rank
# (scripts/rank_sim.py), interleaved twice, each in a fresh process.
# usage: scripts/lib_ab_small.sh "label:lib/path.so" "label2:" ...   ("label:" = lib/libtneqhip.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/lib_ab_small.jsonl
L=quantum_circuits_symmetry_breaking_based_on_tneq-qc_amd/lib
for rep in 1 2; do
  for spec in "$@"; do
    l=${spec%%:*}; p=${spec#*:}
    E=""; [ -n "$p" ] && E="TNEQHIP_LIB=$PWD/$L/$p"
    r=$(env $E timeout -k 10 150 python3 scripts/rank_sim.py C4 2>/dev/null | tail -1) || exit 3
    echo "{\"lib\": \"$l\", \"what\": \"C4 N8 rank\", \"ms\": $(echo $r | python3 -c 'import json,sys; print(json.load(sys.stdin)["rank_ms_N8"])')}" | tee -a $OUT
    for C in C2 C3; do
      b=$(env $E timeout -k 10 120 python3 bench.py --config $C --no-cpu-baseline --no-c5 --no-alt --no-other --steps 100 --warmup 10 2>/dev/null | tail -1) || exit 2
      echo "{\"lib\": \"$l\", \"what\": \"$C\", \"ms\": $(echo $b | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')}" | tee -a $OUT
    done
  done
done
