"""The graph-captured training step (bench.py --config train, its default on one GPU) against
the same step run eagerly.

Reference: the training step of scenedino/training/base_trainer.py:206-257 (sampler ->
forward under autocast -> loss -> backward -> optimizer step), here as bench.train_setup's
body: PatchRaySampler device rays (sd_patch_rays) -> NeRFRenderer / BTSNet training path ->
loss -> backward into the grid leaf and the ResnetFC head -> fused Adam.

Round 4 saw a host segfault when capturing that step after an eager warm-up step on the
legacy default stream: BTSNet's grid cache held a view of the grid leaf with a
grad_fn, which kept the leaf's AccumulateGrad node -- created on the default stream by the
eager step -- alive into the capture, so the autograd engine made the default stream wait on
the capture stream.  The cache now holds a detached view; this test replays the crash
sequence (eager step on the default stream, then capture) and checks the replayed graph
against eager steps on the same patches, jitter and optimizer state.  (Written in round 5,
it also found that the fused training MLP's packed weights were cached by tensor version,
which torch's fused Adam does not bump: the replays used stale weights.)
"""
import os
import sys
import warnings

import pytest
import torch

from _helpers import rel_l2

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _opt_state(opt, params):
    return [{k: v.clone() for k, v in opt.state[p].items()} for p in params]


def _restore(params, values, opt, states):
    with torch.no_grad():
        for p, v in zip(params, values):
            p.copy_(v)
        for p, st in zip(params, states):
            for k, v in st.items():
                opt.state[p][k].copy_(v)


@pytest.mark.parametrize("offset_pose", [False, True])
def test_graphed_training_step_matches_eager(offset_pose):
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import bench
    dev = torch.device("cuda:0")
    ts = bench.train_setup(dev, NB=2, RB=512, offset_pose=offset_pose, capturable=True)
    params = list(ts.head.parameters())
    draw = lambda: ts.sampler.draw(ts.images, ts.dino_gt_map)  # noqa: E731 (host patches)
    slot = torch.empty(draw().shape, dtype=torch.int32, device=dev)

    # warm-up on a side stream (the capture recipe) ...
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(2):
            slot.copy_(draw().to(dev))
            ts.body(slot)
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize()
    # ... and an eager step on the default stream right before the capture: round 4's crash
    slot.copy_(draw().to(dev))
    ts.body(slot)
    torch.cuda.synchronize()

    graph = torch.cuda.CUDAGraph()
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        with torch.cuda.graph(graph):
            loss_g = ts.body(slot).detach()  # (no autograd graph kept alive past the step)
    torch.cuda.synchronize()
    mism = [str(w.message) for w in caught if "AccumulateGrad" in str(w.message)]
    assert not mism, mism[0]
    grads_g = [p.grad for p in params]  # the graph's gradient buffers (its memory pool)
    leaf_g = ts.leaf.grad
    assert leaf_g is not None and all(g is not None for g in grads_g)

    for rep in range(2):
        slot.copy_(draw().to(dev))
        p0 = [p.detach().clone() for p in params]
        s0 = _opt_state(ts.opt, params)
        graph.replay()
        torch.cuda.synchronize()
        zj = ts.zj.clone()  # the jitter drawn inside the replay
        G = [g.clone() for g in grads_g]
        LG = leaf_g.clone()
        P1 = [p.detach().clone() for p in params]
        s1 = _opt_state(ts.opt, params)
        L1 = float(loss_g)
        assert all(not torch.equal(a, b) for a, b in zip(p0, P1)), "replay did not step Adam"

        # the same step eagerly: same patches, jitter and optimizer state
        _restore(params, p0, ts.opt, s0)
        ts.zj.copy_(zj)
        loss_e = ts.body(slot, draw_jitter=False)
        torch.cuda.synchronize()
        assert abs(float(loss_e) - L1) <= 1e-6 * max(1.0, abs(L1)), (rep, float(loss_e), L1)
        for i, (p, g) in enumerate(zip(params, G)):
            assert rel_l2(p.grad, g) <= 1e-6, (rep, "head grad", i)
            assert rel_l2(p.detach(), P1[i]) <= 1e-7, (rep, "head param", i)
        # the grid gradient accumulates with f32 atomics: equal up to summation order
        assert rel_l2(ts.leaf.grad, LG) <= 1e-5, (rep, "grid grad")
        assert float(LG.abs().sum()) > 0
        # continue from the graph's own state
        _restore(params, P1, ts.opt, s1)
