"""BlockPipeline (sampling.py): many amplitude blocks of one network with several plans in flight.
Every block equals the oracle's contraction of that block (circuits.with_batch: other fixed bits);
pipelined steps give the same amplitudes as one-at-a-time runs."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_blocks_match_the_oracle(dev):
    import torch
    from oracle.contract_ref import contract_sliced
    from tneq_qc_amd.circuits import BrickWall, amplitude_task, with_batch
    from tneq_qc_amd.sampling import BlockPipeline
    t = amplitude_task(BrickWall(12, 6, 2), list(range(4, 8)), cut=6, n_slice=2, defer=(2, 2))
    blocks = [0, 3, 5, 9, 130]
    pipe = BlockPipeline(t, blocks, inflight=2, device=dev)
    got = pipe.run()
    for b, g in zip(blocks, got):
        tb = with_batch(t, b)
        ref = contract_sliced(tb.eq, tb.operands, tb.sliced, tb.path)
        assert np.abs(g.numpy() - ref).max() <= 2e-5 * np.abs(ref).max(), b


def test_pipelined_c4_blocks_equal_single_runs(dev):
    import torch
    from tneq_qc_amd.circuits import config_task, with_batch
    from tneq_qc_amd.expression import HipContractExpression
    from tneq_qc_amd.sampling import BlockPipeline
    t = config_task("C4")
    blocks = [0, 1, 2, 3]
    pipe = BlockPipeline(t, blocks, inflight=2, device=dev)
    outs = []
    for k in range(len(blocks)):
        o = pipe.step()
        if k % 2 == 1:   # both slots' blocks enqueued: keep their results before the slots rerun
            pipe.synchronize()
            outs += [pipe.slots[0][3].cpu().numpy().copy(), pipe.slots[1][3].cpu().numpy().copy()]
    e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
    for b, got in zip(blocks, outs):
        tb = with_batch(t, b)
        ops = [torch.from_numpy(x).to(dev, torch.complex64) for x in tb.operands]
        ref = e(*ops).cpu().numpy()
        assert np.abs(got - ref).max() <= 2e-5 * np.abs(ref).max(), b
    assert not np.allclose(outs[0], outs[1])   # other blocks, other amplitudes
