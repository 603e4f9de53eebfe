#!/bin/bash
# Round-2 GPU session 65: PMC passes over the boundary GEMM as the bench now launches it (4 slice
# lanes: one batch-4 launch per 4 slices, no split-K), summarized into profiles/pmc_gemm_f16_r02.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/pmc_gemm_f16.sh && python3 scripts/pmc_gemm_json.py gpurun_out gpurun_out/pmc_gemm_f16_r02k.json f16 4 1
