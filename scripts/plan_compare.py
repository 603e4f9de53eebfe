import os, sys; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sys, torch, tneq_qc_amd, re
from tneq_qc_amd.circuits import amplitude_task, BrickWall
from tneq_qc_amd.einsum import path_info
from tneq_qc_amd.expression import HipContractExpression
cfg = sys.argv[1]; tile = int(sys.argv[2])
if cfg == "C4":
    t = amplitude_task(BrickWall(53, 20, 0), list(range(17, 37)), cut=27, n_slice=3, tile=tile)
else:
    t = amplitude_task(BrickWall(40, 16, 0), list(range(12, 28)), cut=20, n_slice=6, tile=tile)
net = t.network()
sl = [net.symbols.index(x) if hasattr(net.symbols,'index') else x for x in t.sliced]
e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
d = e.plan(torch.complex64).describe()
once = [l for l in d.split('\n') if l.startswith('[once]')]
sl_ = [l for l in d.split('\n') if l.startswith('[slice]')]
sched = [l for l in d.split('\n') if l.startswith('# once')]
print("sliced", t.sliced, "once ops", len(once), "slice ops", len(sl_), "once launches", len(sched))
for l in sl_: print(l[:200])
big = [l for l in once if 'chunks=1 ' not in l and 'chunks=2 ' not in l]
print("once ops with >2 chunks:", len(big))
for l in big[:60]: print(l[:170])
info = path_info(net, t.path, [net.symbols.index(x) for x in t.sliced])
print("est_1 %.3f ms est_8 %.3f ms once %.3f ms slice %.3f ms" % (info.est_seconds*1e3, info.est_ranks(8)*1e3, info.t_once*1e3, info.t_slice*1e3))
