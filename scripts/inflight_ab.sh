cd $GRAFT_REPO_ROOT
for spec in "def:" "mc64:TQ_S2_MINCHUNKS=64" "mc256:TQ_S2_MINCHUNKS=256" "mc32:TQ_S2_MINCHUNKS=32" "lc5:TQ_S2_LC=5" "cap2:TQ_S2_CAP=2" "def2:"; do
  label=${spec%%:*}; envs=${spec#*:}
  r=$(env $envs timeout -k 10 120 python3 probes/inflight.py C4 1 2 2>/dev/null | grep inflight | tr '\n' ' ') || exit 1
  echo "$label $r"
done
