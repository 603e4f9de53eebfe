#!/bin/bash
# Round-2 GPU session 63: sweep2 phase timing of one C4 execute, tables phase split (development build with
# -DTQ_S2_TIMING made on the box, in the box's copy only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
(cd quantum_circuits_symmetry_breaking_based_on_tneq-qc_amd/csrc && make clean > /dev/null && make -j16 EXTRA=-DTQ_S2_TIMING > /dev/null 2>&1) || exit 5
scripts/gpu_check.sh \
  "st63 200 python scripts/sweep_timing.py C4"
