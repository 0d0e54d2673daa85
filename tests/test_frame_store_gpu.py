"""Frame de-duplicated replay (rth_replay_frames_attach / push_frames, the
gather's frame-stack columns): each actor frame enters an HBM frame store once, rows keep
their s0 / s1 stacks as frame ids, the gather assembles the stacks.  Through the Ape-X loop
-- with many episode ends (p_done = 0.25: reset stacks, and the NStepAdder's terminal-bootstrap
rows whose s1 is the terminal stack, reth/reth/utils/nstep_adder.py:14-24) and both the FIFO
and the frame ring wrapping -- every sampled stack, every replay row and every learner update
are bit-identical to the full-row uint8 storage the reference's layout corresponds to
(test/apex-dqn/worker.py:44-51 stores both stacks of every row)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


# the comparison needs a run-to-run deterministic learner: the default conv2 / conv3 weight
# gradients (rth_conv_wgrad_f32, fixed-order partial sums) are; MIOpen's solvers differ in the
# last bits run to run (scripts/diag_fstore.py: the only divergence of the two loops before r04
# was the parameters after the first few updates, on identical batches)


def _run(dev, frame_store, graph, iters=150, env="synthetic", bound="hard", frame_ids=False):
    from reth_amd.apex import ApexConfig, ApexDQN
    from reth_amd.replay import FrameStacks

    cfg = ApexConfig(n_actors=16, capacity=1024, batch_size=32, sample_start=64, p_done=0.25, seed=6,
                     hip_graph=graph, send_weights_interval=3, recv_weights_interval=4, update_target_interval=5,
                     frame_store=frame_store, env=env, frame_store_bound=bound, frame_ids=frame_ids)
    ax = ApexDQN(cfg, device=dev)
    for _ in range(iters):
        ax.iteration()
    torch.cuda.synchronize()
    assert (ax._graphs is not None) == graph
    rep = ax.replay
    size = rep.info()[0]
    s, m, v = rep.tree.export()
    cols = rep.gather(torch.arange(size, device=dev))
    assert all(isinstance(c, FrameStacks) == (frame_ids and k in (0, 3)) for k, c in enumerate(cols))
    cols = [c.stacks() if isinstance(c, FrameStacks) else c for c in cols]
    params = torch.cat([p.detach().flatten() for p in ax.solver._params]).cpu()
    out = dict(tree=[s.cpu(), m.cpu(), v.cpu()], cols=[c.cpu() for c in cols], params=params, info=rep.info(),
               frames=ax.actors.frames.cpu(), updates=ax.updates)
    if frame_store:
        out["head"] = int(rep.frame_head)
        out["F"] = rep.frames.shape[0]
        out["sid_table"] = rep.column_storage(0).cpu()
    ax.close()
    return out


@pytest.mark.parametrize("graph,bound", [(False, "expected"), (True, "hard")])
def test_frame_store_loop_bit_identical_to_full_rows(dev, graph, bound):
    """both store sizes: "hard" (the default: 2 frames per actor step, no row's frames ever
    overwritten) and "expected" (p_done's rate; p_done = 0.25 i.i.d. here)"""
    iters = 230 if bound == "hard" else 150  # enough frames to wrap the larger ring too
    full = _run(dev, False, graph, iters=iters)
    fs = _run(dev, True, graph, iters=iters, bound=bound)
    assert full["info"] == fs["info"] and full["updates"] == fs["updates"] > 50
    assert fs["info"][0] == 1024 and fs["head"] > fs["F"], "the FIFO and the frame ring must both have wrapped"
    names = ["s0", "a", "r", "s1", "done"]
    for name, x, y in zip(names, full["cols"], fs["cols"]):
        assert torch.equal(x, y), (name, int((x != y).sum()))
    for x, y in zip(full["tree"], fs["tree"]):
        assert torch.equal(x, y)
    assert torch.equal(full["frames"], fs["frames"])
    assert torch.equal(full["params"], fs["params"])  # the learner saw the same batches
    done = fs["cols"][4].numpy() != 0
    assert done.any() and (~done).any()


@pytest.mark.parametrize("graph", [False, True])
def test_frame_ids_loop_bit_identical(dev, graph):
    """frames in place (ApexConfig.frame_ids): the learner's batches are frame ids and conv1
    (forward, weight gradient, the target network's forward) reads the frames from the store --
    every update bit-identical to the loop whose gather assembles the stacks"""
    fs = _run(dev, True, graph, iters=150)
    fi = _run(dev, True, graph, iters=150, frame_ids=True)
    assert fs["info"] == fi["info"] and fs["updates"] == fi["updates"] > 50
    for x, y in zip(fs["cols"], fi["cols"]):
        assert torch.equal(x, y)
    assert torch.equal(fs["params"], fi["params"])


def test_frame_store_atari_env(dev):
    """the Atari env mode (device preprocessing, reset screens) into the frame store"""
    full = _run(dev, False, True, iters=60, env="atari")
    fs = _run(dev, True, True, iters=60, env="atari")
    for x, y in zip(full["cols"], fs["cols"]):
        assert torch.equal(x, y)
    assert torch.equal(full["params"], fs["params"])


def test_frame_store_prefill_and_footprint(dev):
    """the prefill's synthetic trajectory: row j's stacks are frames j .. j+3 and j+3 .. j+6 of
    it; the store holds capacity (1 + reset headroom) frames with the "expected" bound, 2
    capacity with the "hard" one: the HBM footprint"""
    from reth_amd.apex import ApexConfig, ApexDQN

    hard = ApexDQN.frame_store_frames(ApexConfig(n_actors=16, capacity=2048, frame_store=True))
    assert hard == 2 * 2048 + 2 * (3 + 16 + 2) * 16 + 16  # + 2 actor_steps_per_update: the sample-ahead window
    cfg = ApexConfig(n_actors=16, capacity=2048, batch_size=32, seed=2, hip_graph=False, frame_store=True,
                     frame_store_bound="expected")
    ax = ApexDQN(cfg, device=dev)
    ax.prefill(cfg.capacity)
    torch.cuda.synchronize()
    rep = ax.replay
    ids = rep.column_storage(0).cpu().numpy()
    base = int(ids[0, 0])
    assert np.array_equal(ids[:, 0], base + np.arange(cfg.capacity))
    rows = torch.tensor([0, 1, 777, cfg.capacity - 1], device=dev)
    s0, _, _, s1, _ = rep.gather(rows)
    s0, s1 = s0.stacks(), s1.stacks()  # frame_ids (the default): the gather wrote the rows' frame ids
    store = rep.frames
    for k, j in enumerate(rows.tolist()):
        assert torch.equal(s0[k], store[base + j:base + j + 4])
        assert torch.equal(s1[k], store[base + j + 3:base + j + 7])
    # ~1 frame per row (+ reset headroom) against 2 x 4 frames per full row
    assert store.shape[0] <= 1.1 * cfg.capacity + 20 * cfg.n_actors + 16
    # the loop runs on from the prefilled state
    for _ in range(8):
        ax.iteration()
    torch.cuda.synchronize()
    assert ax.updates > 0
    ax.close()
