"""End-to-end Ape-X on one GPU at a small size: actors -> HBM replay -> learner -> weights,
plus the graft smoke entry point."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fused", [True, False])
def test_apex_small_end_to_end(dev, fused):
    from reth_amd.apex import ApexConfig, ApexDQN

    cfg = ApexConfig(n_actors=16, capacity=4096, batch_size=32, sample_start=64, send_weights_interval=5,
                     recv_weights_interval=8, update_target_interval=10, p_done=0.05, seed=1, fused_actor=fused)
    ax = ApexDQN(cfg, device=dev)
    for _ in range(60):
        ax.iteration()
    torch.cuda.synchronize()
    size, tail, cnt, calls, steps = ax.replay.info()
    assert steps == ax.updates and calls == ax.updates + 1  # one batch sampled ahead
    lag = 1 if fused else 0  # fused: a step's rows are prioritised and appended one step later
    assert size == 16 * (60 - cfg.n_step - lag) and ax.env_steps == 16 * 60
    assert ax.updates > 40 and ax.slot.version == ax.updates // 5
    assert ax.subscriber.loaded_version > 0
    assert all(torch.isfinite(p).all() for p in ax.solver.q_network.parameters())
    # the replay's last rows are what the actors emitted (the previous step's, when fused)
    act = ax.actors
    rows = act._sets[(act.pushes - 2) % 2] if fused else act._rowset_of_attrs()
    out = ax.replay.gather(torch.arange(tail - 16, tail, device=dev))
    assert torch.equal(out[1], rows.a) and torch.equal(out[2], rows.r)
    assert torch.equal(out[0], act.frames[rows.s0].float())
    assert torch.equal(out[3], act.frames[rows.s1].float())
    ax.close()


def test_graph_replay_matches_eager(dev):
    """HIP-graph replay of the compute blocks keeps every replay/tree op, counter and Philox
    stream of the eager schedule: identical replay state (lr = 0 keeps the networks fixed, so
    MIOpen's atomic weight-gradient reductions cannot make the two runs diverge)"""
    from reth_amd.apex import ApexConfig, ApexDQN

    def run(graph):
        cfg = ApexConfig(n_actors=16, capacity=1024, batch_size=32, sample_start=64, learning_rate=0.0,
                         p_done=0.05, seed=4, hip_graph=graph, send_weights_interval=3,
                         recv_weights_interval=4, update_target_interval=5)
        ax = ApexDQN(cfg, device=dev)
        for _ in range(40):
            ax.iteration()
        torch.cuda.synchronize()
        assert (ax._graphs is not None) == graph
        s, m, v = ax.replay.tree.export()
        cols = ax.replay.gather(torch.arange(ax.replay.info()[0], device=dev))
        out = [s.cpu(), m.cpu(), v.cpu()] + [c.cpu() for c in cols]
        info = ax.replay.info()
        ax.close()
        return out, info

    a, ia = run(False)
    b, ib = run(True)
    assert ia == ib
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_probed_learner_graph_matches_unprobed(dev):
    """the bench's probe sets (a second copy of the actor and learner graphs, cut at the
    launches it times live -- the actor tail, conv2 + conv3, the TD/heads backward, clip+Adam --
    issued eagerly between the parts, each between conv_probe(tag) / conv_probe(tag + "_end"))
    change no result: identical replay state to the unprobed graphs, also when the probe sets
    replay only in a window (the bench's headline window replays the uncut graphs, its probe
    window the cut ones), and every probed iteration reports each launch once"""
    from reth_amd.apex import ApexConfig, ApexDQN

    def run(probe, window=None):
        cfg = ApexConfig(n_actors=16, capacity=1024, batch_size=32, sample_start=64, learning_rate=0.0,
                         p_done=0.05, seed=5, hip_graph=True, send_weights_interval=3,
                         recv_weights_interval=4, update_target_interval=5, extra={"probe_conv2": probe})
        ax = ApexDQN(cfg, device=dev)
        tags, probed = [], 0
        for i in range(40):
            on = window is None or window[0] <= i < window[1]
            ax.conv_probe = tags.append if on else None
            ax.iteration()
            probed += int(on and ax._graphs is not None)  # the capture iteration replays too
        torch.cuda.synchronize()
        assert ax._graphs is not None
        s, m, v = ax.replay.tree.export()
        cols = ax.replay.gather(torch.arange(ax.replay.info()[0], device=dev))
        out = [s.cpu(), m.cpu(), v.cpu()] + [c.cpu() for c in cols]
        info, updates = ax.replay.info(), ax.updates
        ax.close()
        return out, info, tags, probed

    import warnings

    a, ia, ta, _ = run(False)
    with warnings.catch_warnings(record=True) as wl:  # no empty graph captured
        warnings.simplefilter("always")
        b, ib, tb, probed = run(True)
    assert not [w for w in wl if "CUDA Graph is empty" in str(w.message)]
    c, ic, tc, probed_c = run(True, window=(20, 30))
    assert ta == []
    per_iter = ["actor_tail", "actor_tail_end", "conv2", "conv2_end", "conv3", "conv3_end", "td_heads_backward",
                "td_heads_backward_end", "clip_adam", "clip_adam_end"]
    assert probed > 0 and tb == per_iter * probed
    assert probed_c == 10 and tc == per_iter * 10
    assert ia == ib == ic
    for x, y, z in zip(a, b, c):
        assert torch.equal(x, y) and torch.equal(x, z)


def test_graph_split_learner_applies_its_own_gradients(dev):
    """with a gradient all-reduce hook the learner is captured in parts cut at the gradient
    buckets (merged heads | convs | heads split + clip + Adam) per variant and batch parity;
    each replayed apply must consume the gradients its own compute parts wrote (Adam's
    exp_avg after one replayed step follows exactly those gradients)"""
    from reth_amd.apex import ApexConfig, ApexDQN

    cfg = ApexConfig(n_actors=16, capacity=1024, batch_size=32, sample_start=64, seed=4, hip_graph=True,
                     dp_hook=True, update_target_interval=3)
    ax = ApexDQN(cfg, device=dev)
    for _ in range(30):
        ax.iteration()
    G = ax._graphs
    assert G is not None and len(G["learn"]) == 4  # (full | pre target pass) x batch parity
    assert all(len(G["learn"][v]) == 3 and len(G["buckets"][v]) == 2 for v in G["learn"])
    ptrs = [{t.data_ptr() for t in G["grads"][v]} for v in G["grads"]]
    assert all(not (ptrs[i] & ptrs[j]) for i in range(4) for j in range(i))
    opt, params = ax.solver.optimizer, ax.solver._params
    seen = set()
    for _ in range(4):  # both parities, both variants
        torch.cuda.synchronize()  # ax runs on its own stream
        v = ax._next_learner_variant()
        seen.add(v)
        before = [opt.state[p]["exp_avg"].clone() for p in params]
        ax.iteration()
        torch.cuda.synchronize()
        coef = min(cfg.clip_value / (float(opt.total_norm[0]) + 1e-6), 1.0)
        for p, mb, g in zip(params, before, G["grads"][v]):
            torch.testing.assert_close(opt.state[p]["exp_avg"], mb + 0.1 * (g * coef - mb), rtol=1e-5, atol=1e-9)
    assert {v[1] for v in seen} == {0, 1} and ("pre", 0) in seen or ("pre", 1) in seen
    ax.close()


def test_prefill_then_learn(dev):
    from reth_amd.apex import ApexConfig, ApexDQN

    cfg = ApexConfig(n_actors=8, capacity=2000, batch_size=64, seed=2)
    ax = ApexDQN(cfg, device=dev)
    ax.prefill(2000, chunk=700)
    assert ax.replay.info()[0] == 2000 and ax.svc.ready()
    for _ in range(5):
        ax.iteration()
    assert ax.updates == 5
    ax.close()


def test_graft_smoke(dev):
    import __graft_entry__

    __graft_entry__.smoke()


def test_graph_replay_learns(dev):
    """with learning on, graph replay runs the whole loop: finite weights, target syncs,
    weights published and reloaded by the actors"""
    from reth_amd.apex import ApexConfig, ApexDQN

    cfg = ApexConfig(n_actors=32, capacity=4096, batch_size=64, sample_start=128, hip_graph=True, seed=5,
                     send_weights_interval=4, recv_weights_interval=6, update_target_interval=7)
    ax = ApexDQN(cfg, device=dev)
    for _ in range(50):
        ax.iteration()
    torch.cuda.synchronize()
    assert ax._graphs is not None and ax.updates == ax.replay.info()[4]
    assert ax.trainer.cur_step == ax.updates and ax.slot.version == ax.updates // 4
    assert ax.subscriber.loaded_version > 0
    assert all(torch.isfinite(p).all() for p in ax.solver.q_network.parameters())
    assert int(ax.actors.t_dev.item()) == ax.actors.t == 50
    # actors: cached-heads (dedup) steps, and full steps after each weights reload
    assert ax.actor_modes.get("dedup", 0) > 0 and ax.actor_modes.get("full", 0) > 0
    ax.close()


@pytest.mark.parametrize("A", [6, 9, 18])
def test_target_pass_precompute_respects_target_syncs(dev, A):
    """overlapped graph mode computes the next batch's target pass on the actor stream
    ("pre" learner graphs) except right after a target sync, where the learner computes it
    itself ("full"); a precomputed pass equals the target network's output on that batch.
    A = 9 is the reference's Ape-X config (BeamRider, test/apex-dqn/config.yaml:8), 18 the
    full Atari set: the captured target / actor graphs must read the synced weights"""
    from reth_amd.apex import ApexConfig, ApexDQN

    cfg = ApexConfig(n_actors=16, capacity=1024, batch_size=32, sample_start=64, seed=5, hip_graph=True,
                     update_target_interval=4, num_actions=A, send_weights_interval=3, recv_weights_interval=4)
    ax = ApexDQN(cfg, device=dev)
    while ax._graphs is None:
        ax.iteration()
    log = []
    for _ in range(16):
        v = ax._next_learner_variant()
        syncs = ax.solver._target_syncs
        ax.iteration()
        torch.cuda.synchronize()
        synced = ax.solver._target_syncs != syncs
        if v[0] == "pre" and not synced:  # the target weights are still the ones it used
            s1 = ax.loader._slots[v[1]][0][3]
            torch.testing.assert_close(ax._graphs["q1t"][v[1]], ax.solver.target_heads(s1), rtol=0, atol=0)
        log.append((v[0], synced))
    assert any(s for _, s in log) and any(v == "pre" for v, _ in log)
    for (_, synced), (v_next, _) in zip(log, log[1:]):
        if synced:
            assert v_next == "full"
    # the actors' frozen heads / packed convs (what the captured actor graphs read) follow the
    # reloaded parameters
    assert ax.subscriber.loaded_version > 0 and int(ax.actors.action.max()) < A
    an = ax.actor_net
    x = ax.actors.frames[:8]
    with torch.no_grad():
        got = an.forward_heads(x)
        want = an.forward_heads(x, merged=an._merged_head_weights(), packed=an.pack_convs())
    assert torch.equal(got, want)
    ax.close()


def test_breakout_shaped_graph_loop(dev):
    """BASELINE configs[2]'s shape at a small scale (A = 4, many actors relative to the replay):
    graph replay with the dedup actor, the fused learner pass and the fused TD + heads kernel;
    the replay keeps the actors' rows and the weights stay finite"""
    from reth_amd.apex import ApexConfig, ApexDQN

    cfg = ApexConfig(n_actors=128, num_actions=4, capacity=8192, batch_size=64, sample_start=256, hip_graph=True,
                     seed=9, p_done=0.01, send_weights_interval=3, recv_weights_interval=5, update_target_interval=6)
    ax = ApexDQN(cfg, device=dev)
    for _ in range(40):
        ax.iteration()
    torch.cuda.synchronize()
    assert ax._graphs is not None and ax.updates == ax.replay.info()[4]
    assert ax.actor_modes.get("dedup", 0) > 0
    assert all(torch.isfinite(p).all() for p in ax.solver.q_network.parameters())
    act = ax.actors
    assert int(act.action.max()) < 4
    size, tail = ax.replay.info()[:2]
    out = ax.replay.gather(torch.arange(tail - 128, tail, device=dev))
    rows = act._sets[(act.pushes - 2) % 2]
    assert torch.equal(out[1], rows.a) and torch.equal(out[0], act.frames[rows.s0])
    ax.close()



def test_overlapped_allreduce_stream_edges():
    """_learner_replay's comm-stream edges, checked with a stream-ordered stand-in for RCCL
    (tests/_stream_edges.py).  Run in a child process with 16 hardware queues: at the box's
    default of 4, HIP maps the loop's streams onto shared queues, which serialises them in
    submission order and would hide a missing edge (measured: the check passes with both
    edges removed at 4 queues and fails at 16)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GPU_MAX_HW_QUEUES="16")
    r = subprocess.run([sys.executable, "-c", "import tests._stream_edges as m; m.main()"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "stream edges OK" in r.stdout
