#!/bin/bash
# r04: sweep2 phase stamps of C2 in its three launch modes (per level / cooperative chain /
# one-workgroup chain of 4-chunk ops), then the C2 A/B of the cooperative chain.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T=$PWD/quantum_circuits_symmetry_breaking_based_on_tneq-qc_amd/lib/libtneqhip_timing.so
TNEQHIP_LIB=$T TQ_S2_COOP=0 timeout -k 10 100 python scripts/sweep_timing.py C2 > gpurun_out/tim_c2_level.txt 2>&1 || exit 2
TNEQHIP_LIB=$T timeout -k 10 100 python scripts/sweep_timing.py C2 > gpurun_out/tim_c2_coop.txt 2>&1 || exit 3
TNEQHIP_LIB=$T TQ_S2_COOP=0 TQ_S2_SEQCH=4 timeout -k 10 100 python scripts/sweep_timing.py C2 > gpurun_out/tim_c2_chain.txt 2>&1 || exit 4
TNEQHIP_LIB=$T timeout -k 10 100 python scripts/sweep_timing.py C3 > gpurun_out/tim_c3.txt 2>&1 || exit 5
scripts/coop_ab.sh TQ_S2_COOP=1 TQ_S2_COOP=0 "TQ_S2_COOP=0 TQ_S2_SEQCH=4" || exit 6
