# HBM traffic of the boundary GEMM (FETCH_SIZE and WRITE_SIZE in separate passes), one rank of N=8
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gemm_c64 --output-format csv -d gpurun_out/pmcg1 -o run -- python3 scripts/rank_sim.py C4 8 > gpurun_out/pmcg1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex gemm_c64 --output-format csv -d gpurun_out/pmcg2 -o run -- python3 scripts/rank_sim.py C4 8 > gpurun_out/pmcg2.log 2>&1 || exit 2
