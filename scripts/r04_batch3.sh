#!/bin/bash
# r04 final pass: secondary-line profiles (C2 / C3 traffic, C5 trace), the GPU suite, the bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
bash scripts/prof_r04_small.sh > gpurun_out/prof_small.log 2>&1 || { echo "prof_small failed"; tail -5 gpurun_out/prof_small.log; exit 1; }
tail -3 gpurun_out/prof_small.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/gputest_r04c.log 2>&1
rc=$?
tail -2 gpurun_out/gputest_r04c.log
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 600 python3 bench.py > gpurun_out/bench_r04c.json 2> gpurun_out/bench_r04c.err
rc2=$?
tail -c 300 gpurun_out/bench_r04c.json
exit $(( rc != 0 ? rc : rc2 ))
