#!/bin/bash
# Round-2 GPU session 1: parity suite, accuracy of the bench path, headline bench, permute roofline,
# rocprof kernel stats of the bench, GEMM MFMA-busy PMC, permute HBM PMC (separate passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "gputests 420 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread" \
  "acc3m 240 python scripts/accuracy_c4.py --out gpurun_out/accuracy.jsonl" \
  "acc4m 240 env TQ_GEMM_3M=0 python scripts/accuracy_c4.py --out gpurun_out/accuracy.jsonl" \
  "bench 300 python bench.py" \
  "permute 300 python scripts/permute_bench.py" \
  "kt 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o run -- python3 bench.py --no-cpu-baseline" \
  "pmcmfma 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex gemm_c64 --output-format csv -d gpurun_out/pmcmfma -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1" \
  "pmcpf 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex permute --output-format csv -d gpurun_out/pmcpf -o run -- python3 scripts/permute_bench.py --ranks 26,28 --dtypes c64,c128 --perms 1 --reps 3" \
  "pmcpw 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex permute --output-format csv -d gpurun_out/pmcpw -o run -- python3 scripts/permute_bench.py --ranks 26,28 --dtypes c64,c128 --perms 1 --reps 3"
