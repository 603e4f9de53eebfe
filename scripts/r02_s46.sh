#!/bin/bash
# Round-2 GPU session 46: what bounds the big per-slice sweep2 launch -- default build, no
# epilogue (TQ_S2_EPI=0), no register blocks, and diagnostic builds without the gate arithmetic
# (-DTQ_S2_DIAG=1) / without HBM stores (-DTQ_S2_DIAG=2); built on the box, in its copy only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sv_$lab -o run -- python3 scripts/sweep_variant.py > gpurun_out/sv_$lab.log 2>&1 || return 1
  python3 scripts/sweep_trace_summary.py gpurun_out/sv_$lab/run_kernel_trace.csv $lab | tee -a gpurun_out/sv_summary.txt
}
rm -f gpurun_out/sv_summary.txt
run default TQ_X=1 && run noepi TQ_S2_EPI=0 && run noblk TQ_S2_BLOCKS=0 || exit 1
mk() { (cd quantum_circuits_symmetry_breaking_based_on_tneq-qc_amd/csrc && touch tq_sweep2.hip && make -j16 EXTRA="$1" > /dev/null 2>&1); }
mk -DTQ_S2_DIAG=1 && run nomac TQ_X=1 || exit 1
mk -DTQ_S2_DIAG=2 && run nostore TQ_X=1 || exit 1
cat gpurun_out/sv_summary.txt
