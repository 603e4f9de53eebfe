#!/bin/bash
# Instruction-cache behaviour of the sweep2 kernel (71.6 KB of gfx950 code for complex64, more
# than the 64-KB instruction cache two CUs share): the available SQC counters, then one PMC pass
# over the C2 bench (every op a latency-bound sweep2 launch).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ic
timeout -s KILL 60 rocprofv3 -L > gpurun_out/ic/avail.txt 2>&1 || true
grep -E "SQC_|SQ_IFETCH|SQ_INSTS_VALU\b|SQ_WAIT_INST_ANY" gpurun_out/ic/avail.txt | head -40 > gpurun_out/ic/avail_sqc.txt || true
B="python3 bench.py --config C2 --no-cpu-baseline --no-c5 --no-alt --no-other --steps 2 --warmup 1"
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_INSTS_VALU --kernel-include-regex sweep2 --output-format csv -d gpurun_out/ic/p1 -o run -- $B > gpurun_out/ic/p1.log 2>&1 || exit 1
python3 scripts/pmc_summary.py sweep2 gpurun_out/ic > gpurun_out/ic/summary.txt 2>&1 || true
