#!/bin/bash
# r04 final pass, second part: the GPU suite and the bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/gputest_r04g.log 2>&1
rc=$?
tail -2 gpurun_out/gputest_r04g.log
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 600 python3 bench.py > gpurun_out/bench_r04g.json 2> gpurun_out/bench_r04g.err
rc2=$?
tail -c 300 gpurun_out/bench_r04g.json
exit $(( rc != 0 ? rc : rc2 ))
