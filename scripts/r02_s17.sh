#!/bin/bash
# Round-2 GPU session 17: list the gfx950 PMC counters; sweep2 stall breakdown on C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
echo "list exit $?"
scripts/gpu_check.sh \
  "pmcw 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex sweep2 --output-format csv -d gpurun_out/pmcw -o run -- python3 scripts/rank_sim.py C4 8"
