#!/bin/bash
# Round-2 GPU session 14: sweep2 with register-held coefficients, byte-offset LDS addressing,
# first-chunk loads before table staging, c128 slots out of scratch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "ctests 400 python -u -m pytest tests/test_contract_gpu.py tests/test_fullsize_gpu.py tests/test_kernels_gpu.py -m gpu -q -rf --timeout 200 --timeout-method thread" \
  "s2t 200 env TNEQHIP_LIB=$PWD/quantum_circuits_symmetry_breaking_based_on_tneq-qc_amd/lib/libtneqhip_s2t.so python scripts/sweep_timing.py C4" \
  "ranksim 200 python scripts/rank_sim.py C4" \
  "bench 300 python bench.py --no-c5"
