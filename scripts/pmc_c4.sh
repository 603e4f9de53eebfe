# PMC passes over the C4 plan (one rank of N=8): the same four passes as pmc_sweep.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/c4pmc1 -o run -- python3 scripts/rank_sim.py C4 8 > gpurun_out/c4pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM --output-format csv -d gpurun_out/c4pmc2 -o run -- python3 scripts/rank_sim.py C4 8 > gpurun_out/c4pmc2.log 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/c4pmc3 -o run -- python3 scripts/rank_sim.py C4 8 > gpurun_out/c4pmc3.log 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/c4pmc4 -o run -- python3 scripts/rank_sim.py C4 8 > gpurun_out/c4pmc4.log 2>&1 || exit 4
