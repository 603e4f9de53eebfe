#!/bin/bash
# Round-4 evidence for the secondary lines: HBM traffic of the C2 / C3 sweep launches (one PMC
# pass per counter, FETCH_SIZE and WRITE_SIZE, over the same bench command the line runs) and a
# kernel trace of the C5 training bench (launches per candidate-step, GPU-busy fraction).
#   gpurun -- 'bash scripts/prof_r04_small.sh' ; python scripts/prof_r04_small_json.py gpurun_out/p04s
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/p04s
O=gpurun_out/p04s
R="--kernel-include-regex sweep --output-format csv"
for C in C2 C3; do
  B="python3 bench.py --config $C --no-cpu-baseline --no-c5 --no-alt --no-other --steps 2 --warmup 1"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE $R -d $O/${C}_f -o run -- $B > $O/${C}_f.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE $R -d $O/${C}_w -o run -- $B > $O/${C}_w.log 2>&1 || exit 2
done
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $O/c5 -o run -- python3 scripts/c5_bench.py --steps 10 --warmup 3 --cpu-steps 0 > $O/c5.log 2>&1 || exit 3
python3 scripts/prof_r04_small_json.py $O
