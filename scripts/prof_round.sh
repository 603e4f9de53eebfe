# Per-round profile of the C4 bench command: kernel-trace stats of the bench run, then one PMC
# pass per counter set over the boundary GEMM, the dense sweep and the sweep2 launches (a short
# bench run each), summarized by scripts/prof_round_json.py into profiles/*_<tag>.json (run that
# locally on the merged gpurun_out/p<tag>).  Usage: scripts/prof_round.sh r04
TAG=${1:-r04}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/p$TAG
O=gpurun_out/p$TAG
B="python3 bench.py --no-cpu-baseline --no-c5 --no-alt --no-other --steps 2 --warmup 1"
R="--kernel-include-regex split_kernel|gemm_planes_kernel|sweepd_kernel|sweep2_kernel --output-format csv"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --no-cpu-baseline --no-c5 --no-alt --no-other > $O/kt.json 2> $O/kt.log || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace $R -d $O/k0 -o run -- $B > $O/k0.log 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT $R -d $O/p1 -o run -- $B > $O/p1.log 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY $R -d $O/p2 -o run -- $B > $O/p2.log 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE $R -d $O/p3 -o run -- $B > $O/p3.log 2>&1 || exit 5
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE $R -d $O/p4 -o run -- $B > $O/p4.log 2>&1 || exit 6
