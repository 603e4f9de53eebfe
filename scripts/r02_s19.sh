#!/bin/bash
# Round-2 GPU session 19: per-pass clocks of the first chunk of every sweep2 op (C4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "s2t 200 env TNEQHIP_LIB=$PWD/quantum_circuits_symmetry_breaking_based_on_tneq-qc_amd/lib/libtneqhip_s2t.so python scripts/sweep_timing.py C4" \
  "s2t0 200 env TQ_S2_BLOCKS=0 TNEQHIP_LIB=$PWD/quantum_circuits_symmetry_breaking_based_on_tneq-qc_amd/lib/libtneqhip_s2t.so python scripts/sweep_timing.py C4"
