# HBM traffic (2*FETCH_SIZE + WRITE_SIZE, separate PMC passes) of the secondary lines: the sweep
# launches of C2, C3, C4 and C4x4 (bench.py --config; CFGS="..." restricts them), and every kernel of the C5 training step
# (scripts/c5_bench.py); summarized by scripts/pmc_traffic_json.py into profiles/pmc_<cfg>_<tag>.json
# (run that locally on the merged gpurun_out/t<tag>).  Usage: scripts/pmc_traffic.sh r05
TAG=${1:-r05}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/t$TAG
O=gpurun_out/t$TAG
for cfg in ${CFGS:-C2 C3 C4 C4x4}; do
  B="python3 bench.py --config $cfg --no-cpu-baseline --no-c5 --no-alt --no-other --steps 2 --warmup 1"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --kernel-include-regex sweep --output-format csv -d $O/${cfg}_$c -o run -- $B > $O/${cfg}_$c.log 2>&1 || exit 1
  done
done
[ "${SKIP_C5:-0}" = 1 ] && exit 0
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/C5_$c -o run -- python3 scripts/c5_bench.py --steps 2 --warmup 1 --cpu-steps 0 > $O/C5_$c.log 2>&1 || exit 2
done
