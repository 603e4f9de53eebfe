# VALU / LDS issue activity of the sweep2 launches in the headline bench (one PMC pass).
# usage: scripts/pmc_valu.sh <tag>   -> gpurun_out/pv<tag>/
TAG=${1:-r06}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pv$TAG
O=gpurun_out/pv$TAG
B="python3 bench.py --no-cpu-baseline --no-c5 --no-alt --no-other --steps 20 --warmup 3"
R="--kernel-include-regex sweep2_kernel --output-format csv"
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE $R -d $O/p1 -o run -- $B > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace $R -d $O/k0 -o run -- $B > $O/k0.log 2>&1 || exit 2
