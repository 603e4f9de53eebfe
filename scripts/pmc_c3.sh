# PMC passes (one counter set per run) over the C3 bench (the per-slice sweep2 launch dominates):
#   gpurun -- 'bash scripts/pmc_c3.sh' ; python scripts/pmc_summary.py sweep2 gpurun_out/c3p
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/c3p
B="python3 bench.py --config C3 --no-cpu-baseline --no-c5 --no-alt --no-other --steps 2 --warmup 1"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/c3p/pmc1 -o run -- $B > gpurun_out/c3p/pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/c3p/pmc3 -o run -- $B > gpurun_out/c3p/pmc3.log 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/c3p/pmc4 -o run -- $B > gpurun_out/c3p/pmc4.log 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM --output-format csv -d gpurun_out/c3p/pmc2 -o run -- $B > gpurun_out/c3p/pmc2.log 2>&1 || exit 2
