#!/bin/bash
# Round-2 GPU session 3: permute with native 16-B vector accesses and full-size tiles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "ktests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_contract_gpu.py tests/test_strategy_gpu.py -m gpu -q -rf --timeout 200 --timeout-method thread" \
  "perm 300 python scripts/permute_bench.py --ranks 20,22,24,26,28 --dtypes c64,c128,f64,f32 --perms 3" \
  "pmcpf 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex permute --output-format csv -d gpurun_out/pmcpf -o run -- python3 scripts/permute_bench.py --ranks 26,28 --dtypes c64,c128 --perms 1 --reps 3" \
  "pmcpw 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex permute --output-format csv -d gpurun_out/pmcpw -o run -- python3 scripts/permute_bench.py --ranks 26,28 --dtypes c64,c128 --perms 1 --reps 3" \
  "pmcps 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-include-regex permute --output-format csv -d gpurun_out/pmcps -o run -- python3 scripts/permute_bench.py --ranks 26,28 --dtypes c64,c128 --perms 1 --reps 3"
