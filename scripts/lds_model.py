import time, torch, tneq_qc_amd, sys
from tneq_qc_amd.circuits import config_task
from tneq_qc_amd.expression import HipContractExpression
for cfg in ['C4','C3','C2']:
  task = config_task(cfg)
  t=time.time()
  expr = HipContractExpression(task.eq, *task.shapes, optimize=task.path, slices=task.sliced)
  plan = expr.plan(torch.complex64)
  dt=time.time()-t
  a=b=0;n=0
  for l in plan.describe().splitlines():
    if 'ldsx' in l:
      x=l[l.index('ldsx=')+5:].split()[0].split('->'); a+=float(x[0]); b+=float(x[1]); n+=1
      if '[slice]' in l: print(cfg, l[:40], l[l.index('ldsx'):])
  print(cfg, "plan %.2fs ops %d mean legacy %.2f new %.2f"%(dt,n,a/n,b/n))
