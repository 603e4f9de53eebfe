"""BlockPipeline (sampling.py): many amplitude blocks of one network, several groups in flight
and several blocks per lockstep group (blocks as lanes: tq_plan_execute_group).  Every block
equals the oracle's contraction of that block (circuits.with_batch: other fixed bits); grouped
and pipelined blocks equal one-at-a-time runs, partial groups included."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("inflight,group", [(2, 1), (1, 3), (2, 2)])
def test_blocks_match_the_oracle(dev, inflight, group):
    from oracle.contract_ref import contract_sliced
    from tneq_qc_amd.circuits import BrickWall, amplitude_task, with_batch
    from tneq_qc_amd.sampling import BlockPipeline
    t = amplitude_task(BrickWall(12, 6, 2), list(range(4, 8)), cut=6, n_slice=2, defer=(2, 2))
    blocks = [0, 3, 5, 9, 130]   # 5 blocks: the last group is partial
    pipe = BlockPipeline(t, blocks, inflight=inflight, group=group, device=dev)
    got = pipe.run()
    assert len(got) == len(blocks)
    for b, g in zip(blocks, got):
        tb = with_batch(t, b)
        ref = contract_sliced(tb.eq, tb.operands, tb.sliced, tb.path)
        assert np.abs(g.numpy() - ref).max() <= 1e-5 * np.abs(ref).max(), b


@pytest.mark.parametrize("inflight,group", [(2, 1), (2, 4)])
def test_pipelined_c4_blocks_equal_single_runs(dev, inflight, group):
    """The benchmarked C4 pipeline (bench.py: `--inflight` x `--group`) against single-block
    executes of the plain expression: 2 x group blocks (every slot once), then one block more
    (a partial group through flush())."""
    import torch
    from tneq_qc_amd.circuits import config_task, with_batch
    from tneq_qc_amd.expression import HipContractExpression
    from tneq_qc_amd.sampling import BlockPipeline
    t = config_task("C4")
    n = inflight * group
    blocks = list(range(n + 1))
    pipe = BlockPipeline(t, blocks, inflight=inflight, group=group, device=dev)
    outs = [pipe.step() for _ in range(n)]
    pipe.wait()
    torch.cuda.current_stream().synchronize()
    got = [o.cpu().numpy().copy() for o in outs]
    last = pipe.step()          # block n: member 0 of slot 0 again, launched by synchronize()
    pipe.synchronize()
    got.append(last.cpu().numpy().copy())
    e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
    for b, g in zip(blocks, got):
        tb = with_batch(t, b)
        ops = [torch.from_numpy(x).to(dev, torch.complex64) for x in tb.operands]
        ref = e(*ops).cpu().numpy()
        assert np.abs(g - ref).max() <= 1e-5 * np.abs(ref).max(), b
    assert not np.allclose(got[0], got[1])   # other blocks, other amplitudes


def test_run_group_refuses_mismatched_members(dev):
    import torch
    from tneq_qc_amd.expression import HipContractExpression, run_group
    rng = np.random.default_rng(0)

    def ops(shapes):
        return [torch.tensor(rng.standard_normal(s) + 1j * rng.standard_normal(s), dtype=torch.complex64,
                             device=dev) for s in shapes]
    e1 = HipContractExpression("ab,bc->ac", (8, 16), (16, 4))
    e2 = HipContractExpression("ab,bc,cd->ad", (8, 16), (16, 4), (4, 2))
    b1 = e1.bind(*ops([(8, 16), (16, 4)]), private_plan=True)
    b2 = e2.bind(*ops([(8, 16), (16, 4), (4, 2)]), private_plan=True)
    with pytest.raises(ValueError):
        run_group([b1, b2], [b1.new_out(), b2.new_out()])
    # the same plan twice is refused (one arena cannot hold two blocks)
    with pytest.raises(ValueError):
        run_group([b1, b1], [b1.new_out(), b1.new_out()])
    # a matching pair runs and equals the single runs
    x, y = ops([(8, 16), (16, 4)]), ops([(8, 16), (16, 4)])
    m1, m2 = e1.bind(*x, private_plan=True), e1.bind(*y, private_plan=True)
    o1, o2 = m1.new_out(), m2.new_out()
    run_group([m1, m2], [o1, o2])
    torch.cuda.synchronize()
    for o, (a, b) in ((o1, x), (o2, y)):
        ref = (a @ b).cpu().numpy()
        assert np.abs(o.cpu().numpy() - ref).max() <= 1e-5 * np.abs(ref).max()
