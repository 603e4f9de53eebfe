#!/bin/bash
# Round-2 GPU session 13: sweep2 with host-built tables: parity, phase timing, PMC on sweep2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "ctests 300 python -u -m pytest tests/test_contract_gpu.py tests/test_fullsize_gpu.py -m gpu -q -rf --timeout 200 --timeout-method thread" \
  "s2t 200 env TNEQHIP_LIB=$PWD/quantum_circuits_symmetry_breaking_based_on_tneq-qc_amd/lib/libtneqhip_s2t.so python scripts/sweep_timing.py C4" \
  "ranksim 200 python scripts/rank_sim.py C4" \
  "pmcs 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU --kernel-include-regex sweep2 --output-format csv -d gpurun_out/pmcs -o run -- python3 scripts/rank_sim.py C4 8"
