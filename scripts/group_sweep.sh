# Same-box A/B of the C4 headline over (group, inflight): blocks per lockstep group x groups in
# flight (bench.py --group / --inflight).  Usage: scripts/group_sweep.sh TAG "g,i g,i ..."
TAG=${1:-r06}
SET=${2:-"1,4 4,1 4,2 8,1 2,4 8,2"}
mkdir -p gpurun_out
for gi in $SET; do
  g=${gi%,*}; i=${gi#*,}
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-c5 --no-alt --no-other --steps 48 --warmup 8 \
      --group $g --inflight $i > gpurun_out/gs_${TAG}_g${g}_i${i}.json 2> gpurun_out/gs_${TAG}_g${g}_i${i}.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],4), 'ms/block', round(d['value']/1e9,3), 'G amp/s', 'lat', round(d['timing']['latency_ms_per_step'],4))" gpurun_out/gs_${TAG}_g${g}_i${i}.json "g=$g i=$i" | tee -a gpurun_out/gs_${TAG}.txt
done
