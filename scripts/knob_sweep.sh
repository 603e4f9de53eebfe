# Same-box A/B of the C4 headline over env knobs x in-flight depth.  Usage:
#   scripts/knob_sweep.sh TAG "label:VAR=v ..." ... (INFL="4 6" env: in-flight depths)
TAG=$1; shift
mkdir -p gpurun_out
for spec in "$@"; do
  label=${spec%%:*}; envs=${spec#*:}
  for i in ${INFL:-4}; do
    env $envs timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-c5 --no-alt --no-other --steps 48 --warmup 8 \
        --inflight $i > gpurun_out/ks_${TAG}_${label}_i$i.json 2> gpurun_out/ks_${TAG}_${label}_i$i.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],4), 'ms/block', 'lat', round(d['timing']['latency_ms_per_step'],4), 'sweep us', d['roofline'].get('avg_launch_us_events'))" gpurun_out/ks_${TAG}_${label}_i$i.json "$label i=$i" | tee -a gpurun_out/ks_${TAG}.txt
  done
done
