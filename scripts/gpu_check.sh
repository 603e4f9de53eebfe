#!/bin/bash
# GPU session driver: each GPU step under its own time limit; stop at the first fault-class exit
# (abort 134, segfault 139, timeout 124/137) — a plain test failure (1) does not stop the run.
# usage: scripts/gpu_check.sh "<label> <seconds> <command...>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for step in "$@"; do
  label=$(echo "$step" | awk '{print $1}')
  secs=$(echo "$step" | awk '{print $2}')
  cmd=$(echo "$step" | cut -d' ' -f3-)
  echo "== $label ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$label.log" 2>&1
  rc=$?
  echo "== $label exit $rc"
  tail -4 "gpurun_out/$label.log"
  case $rc in
    124|134|137|139) echo "== fault-class exit $rc: stopping"; exit $rc ;;
  esac
done
