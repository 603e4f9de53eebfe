#!/bin/bash
# Round-2 GPU session 28: f16 split GEMM memory-path counters (TCP request latency / stalls).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
R="--kernel-include-regex split_kernel --output-format csv"
B="python3 scripts/gemm_c64_bench.py --bench-shape"
scripts/gpu_check.sh \
  "m1 90 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_LATENCY_sum GRBM_GUI_ACTIVE $R -d gpurun_out/m1 -o run -- $B" \
  "m2 90 rocprofv3 --pmc TCP_TA_TCP_STATE_READ_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr TA_TA_BUSY_sum $R -d gpurun_out/m2 -o run -- $B" \
  "m3 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum $R -d gpurun_out/m3 -o run -- $B"
