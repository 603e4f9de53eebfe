#!/bin/bash
# r04 measurement batch: loss / C5 tests, C5 loss + one-graph A/B, GEMM static-priority A/B,
# then the per-round profile (each step under its own time limit; stops on a fault-class exit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
scripts/gpu_check.sh "loss 400 python -u -m pytest tests/test_loss_gpu.py tests/test_c5_parity_gpu.py tests/test_c5_streams_gpu.py -x -q --timeout 300 --timeout-method thread" || exit 1
grep -q " passed" gpurun_out/loss.log || exit 1
c5() { timeout -k 10 150 env $1 python3 scripts/c5_bench.py --steps 30 --warmup 5 --cpu-steps 0 $2 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(\"c5 [$1 $2]\", round(d[\"value\"]), round(d[\"ms_per_step\"],3), d.get(\"host_issue_ms_per_step\"))"; }
for r in 1 2; do
  c5 "C5_TORCH_LOSS=1" "" || exit 2
  c5 "C5_TORCH_LOSS=0" "" || exit 2
  c5 "C5_TORCH_LOSS=0" "--one-graph" || exit 2
done
scripts/ab_env.sh "p0:TQ_GEMM_PRIO=0" "p1:TQ_GEMM_PRIO=1" "l8:TQ_SLICE_LANES=8 TQ_LANE_ARENA_MB=16384" "p0b:TQ_GEMM_PRIO=0" "p1b:TQ_GEMM_PRIO=1" "l8b:TQ_SLICE_LANES=8 TQ_LANE_ARENA_MB=16384" || exit 3
scripts/prof_round.sh r04
