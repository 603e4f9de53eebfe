#!/bin/bash
# Round-2 GPU session 7: SGDG kernel parity; sweep2 phase timing (instrumented library) after
# staging the gate tensors with the descriptor.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "optim 300 python -u -m pytest tests/test_optim_gpu.py -m gpu -q -rf --timeout 200 --timeout-method thread" \
  "s2t 200 env TNEQHIP_LIB=$PWD/quantum_circuits_symmetry_breaking_based_on_tneq-qc_amd/lib/libtneqhip_s2t.so python scripts/sweep_timing.py C4"
