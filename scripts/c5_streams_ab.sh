cd $GRAFT_REPO_ROOT
for s in 8 4 2 8 4 1; do
  timeout -k 10 200 python3 scripts/c5_bench.py --steps 20 --warmup 5 --cpu-steps 0 --streams $s > gpurun_out/c5s_$s.json 2> gpurun_out/c5s_$s.err || exit 1
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/c5s_$s.json') if l.startswith('{')][-1]); print('streams $s', d.get('streams'), round(d['value'],1), round(d['ms_per_step'],3))"
done
