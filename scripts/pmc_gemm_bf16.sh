# PMC passes (one counter set per run) over the C4 boundary GEMM in bench.py (bf16-split kernel),
# plus the kernel-trace stats of the same bench command; summarized by scripts/pmc_gemm_json.py
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
B="python3 bench.py --no-cpu-baseline --no-c5 --no-alt --no-other --steps 2 --warmup 1"
R="--kernel-include-regex gemm_c64 --output-format csv"
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT $R -d gpurun_out/pmcx1 -o run -- $B > gpurun_out/pmcx1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE $R -d gpurun_out/pmcx2 -o run -- $B > gpurun_out/pmcx2.log 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE $R -d gpurun_out/pmcx3 -o run -- $B > gpurun_out/pmcx3.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktx -o run -- python3 bench.py --no-cpu-baseline --no-c5 --no-alt --no-other > gpurun_out/ktx.log 2>&1 || exit 4
