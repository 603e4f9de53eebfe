#!/bin/bash
# Round-2 GPU session 49: chunk width of the latency-bound small sweep ops (hoisted chain):
# TQ_S2_MINCHUNKS / TQ_S2_MINLC variants, whole-execute time and sweep time per execute.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/sv_summary.txt
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sv_$lab -o run -- python3 scripts/sweep_variant.py > gpurun_out/sv_$lab.log 2>&1 || return 1
  echo "$lab $(grep ms_per_execute gpurun_out/sv_$lab.log)" | tee -a gpurun_out/sv_summary.txt
  python3 scripts/sweep_trace_summary.py gpurun_out/sv_$lab/run_kernel_trace.csv $lab 14 | tee -a gpurun_out/sv_summary.txt
}
run c256_2 TQ_X=1 && run c512_1 TQ_S2_MINCHUNKS=512 TQ_S2_MINLC=1 && run c1024_0 TQ_S2_MINCHUNKS=1024 TQ_S2_MINLC=0 \
  && run c512_0 TQ_S2_MINCHUNKS=512 TQ_S2_MINLC=0 && run c256_0 TQ_S2_MINCHUNKS=256 TQ_S2_MINLC=0 || exit 1
