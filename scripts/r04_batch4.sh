#!/bin/bash
# r04 final pass after the sweep2 pass-head change: C4 profile (kernel stats + PMC passes), the
# GPU suite, the bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
bash scripts/prof_round.sh r04d > gpurun_out/prof_r04d.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_r04d.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/gputest_r04d.log 2>&1
rc=$?
tail -2 gpurun_out/gputest_r04d.log
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 600 python3 bench.py > gpurun_out/bench_r04d.json 2> gpurun_out/bench_r04d.err
rc2=$?
tail -c 300 gpurun_out/bench_r04d.json
exit $(( rc != 0 ? rc : rc2 ))
