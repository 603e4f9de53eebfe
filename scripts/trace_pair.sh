# Kernel traces of the headline phase alone for several (group, inflight) settings, summarised.
# Usage: scripts/trace_pair.sh TAG "g,i g,i ..."
TAG=${1:-r06}
SET=${2:-"1,1 4,1"}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tr_$TAG
for gi in $SET; do
  g=${gi%,*}; i=${gi#*,}
  O=gpurun_out/tr_$TAG/g${g}_i${i}
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 scripts/headline_trace.py --group $g --inflight $i --steps 16 --warmup 8 > $O.json 2> $O.log || exit 1
  f=$(find $O -name "*kernel_trace.csv" | head -1)
  python3 scripts/regime_summary.py $f 16 > $O.summary.json || exit 2
done
