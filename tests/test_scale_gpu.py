"""BASELINE configs at their own sizes.

* The sum-tree through the Ape-X loop's real launch shape at Pong (C = 1,000,000, depth 20:
  256 appended rows + the previous update's 512 deferred priorities per launch) and at
  Breakout (C = 4,000,000, depth 22: 2,048 + 512), wrapping the FIFO, bit-exact against the
  oracle's sequential tree (sum / min / val, then sampled indices and IS weights under
  recorded uniforms).  Reference: reth_buffer/reth_buffer/utils/sumtree.py:5-79,
  per_sampler.py:16-28, fifo_policy.py:11-18, test/apex-dqn/config.yaml.
* Bulk and skewed updates that take the subtree pass's multi-round and entry-overflow
  paths (many keys in one workgroup; a depth-24 tree whose subtrees hold 8,191 nodes).
* ApexDQN at configs[1] (256 actors, 1 M rows, B = 512) and configs[2] (2,048 actors,
  A = 4, 4 M rows) sizes: counters, replay rows == the actors' rows, tree invariants, and
  graph replay == eager at lr = 0.
"""
import gc

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _no_top_pass_timeouts():
    """every tree update's concurrent top pass found its subtree workgroups done within its
    bounded wait (a timeout would leave the levels above S stale: ADVICE r05)"""
    from reth_amd.replay import tree_update_timeouts

    before = tree_update_timeouts()
    yield
    torch.cuda.synchronize()
    assert tree_update_timeouts() == before, "tree-update top pass timed out"


def _export(tree):
    s, m, v = tree.export()
    torch.cuda.synchronize()
    return s.cpu().numpy(), m.cpu().numpy(), v.cpu().numpy()


def _assert_tree_equal(tree, o):
    s, m, v = _export(tree)
    assert np.array_equal(v, o.val), "val"
    assert np.array_equal(s, o.sum), "sum"
    assert np.array_equal(m, o.min_), "min"


@pytest.mark.parametrize("passes", ["1", "2", "0"])
@pytest.mark.parametrize("cap,n_app,steps", [(1_000_000, 256, 40), (4_000_000, 2048, 40)])
def test_loop_shaped_tree_vs_oracle(dev, orc, cap, n_app, steps, passes, monkeypatch):
    """prefill to near capacity, then per step one merged launch: the previous learner
    update's 512 priorities (deferred, step=True) + n_app appended rows, wrapping the FIFO;
    passes = 2: the two-pass subtree update of deep trees (RTH_TREE_PASSES), 0: the default rule
    (two passes from 1,536 keys of one launch)"""
    monkeypatch.setenv("RTH_TREE_PASSES", passes)
    from reth_amd.replay import Column, HbmReplay

    B = 512
    rng = np.random.default_rng(cap + n_app)
    rep = HbmReplay(cap, [Column((), torch.int64)], alpha=0.5, beta="0.4,1,2000000", device=dev, seed=1)
    o = orc.Tree(cap)
    tail = 0
    pre = cap - n_app * (steps // 2)  # the FIFO wraps half way through the loop
    chunk = 1 << 18
    for st in range(0, pre, chunk):
        m = min(chunk, pre - st)
        td = rng.random(m, dtype=np.float32)
        rep.append([torch.arange(st, st + m, device=dev)], torch.as_tensor(td, device=dev))
        slots, tail = orc.fifo_indices(cap, tail, m)
        o.update(slots, orc.per_normalize(td, 0.5).astype(np.float64))
    for k in range(steps):
        idx = rng.integers(0, min(cap, pre + k * n_app), B)
        idx[:8] = idx[8:16]  # duplicates inside one update: last writer wins
        td_upd = rng.random(B, dtype=np.float32)
        td_upd[:4] = 0.0
        rep.update_priorities(torch.as_tensor(idx, device=dev), torch.as_tensor(td_upd, device=dev), step=True,
                              deferred=True)
        td_app = rng.random(n_app, dtype=np.float32)
        rep.append([torch.arange(n_app, device=dev)], torch.as_tensor(td_app, device=dev))
        o.update(idx, orc.per_normalize(td_upd, 0.5).astype(np.float64))
        slots, tail = orc.fifo_indices(cap, tail, n_app)
        o.update(slots, orc.per_normalize(td_app, 0.5).astype(np.float64))
    torch.cuda.synchronize()
    assert rep.info()[1] == tail and rep.info()[4] == steps
    _assert_tree_equal(rep.tree, o)
    u = rng.random(B)
    gi, gv = rep.tree.sample(B, uniforms=u)
    oi, ov = o.sample(u)
    assert np.array_equal(gi.cpu().numpy(), oi) and np.array_equal(gv.cpu().numpy(), ov)
    # the shard's own PER sample: beta stepped once per update message
    _, idx_s, isw = rep.sample(B, uniforms=u)
    beta = 0.4 + (1.0 - 0.4) * steps / 2000000
    assert np.array_equal(idx_s.cpu().numpy(), oi)
    np.testing.assert_allclose(isw.cpu().numpy(), orc.per_is_weights(ov, o.min(), beta), rtol=1e-12, atol=0)


def test_bulk_update_many_rounds(dev, orc):
    """one call with ~1,200 keys per subtree workgroup (two gather rounds each) and heavy
    duplication, then a FIFO-shaped bulk append of 2^17 rows"""
    from reth_amd.replay import SumTree

    rng = np.random.default_rng(5)
    cap = (1 << 18) + 12345
    t, o = SumTree(cap, dev), orc.Tree(cap)
    idx = rng.integers(0, cap, 300_000)
    dup = idx[1::7]
    idx[0:7 * len(dup):7] = dup
    w = rng.random(len(idx))
    w[rng.random(len(idx)) < 0.02] = 0.0
    t.update(idx, w)
    o.update(idx, w)
    _assert_tree_equal(t, o)
    idx = np.arange(1 << 17) + 77
    w = rng.random(len(idx))
    t.update(idx, w)
    o.update(idx, w)
    _assert_tree_equal(t, o)


def _subtree_ids(root, level, cap, maxd, rng, n):
    """n random node ids inside the subtree of `root` (a node at `level`), all depths"""
    out = []
    while len(out) < n:
        d = int(rng.integers(level, maxd + 1))
        lo = ((root + 1) << (d - level)) - 1
        hi = min(((root + 2) << (d - level)) - 2, cap - 1)
        if lo <= hi:
            out.append(int(rng.integers(lo, hi + 1)))
    return np.array(out, dtype=np.int64)


def test_skewed_keys_entry_overflow(dev, orc):
    """C = 2^24 + 5 (depth 25): 3,000 random keys inside ONE level-11 subtree (8,191+ nodes)
    land in one workgroup whose touched (node, level) entries exceed LDS -- the round is
    re-gathered with fewer keys -- plus keys in the dense top and a neighbouring subtree"""
    from reth_amd.replay import SumTree

    rng = np.random.default_rng(8)
    cap = (1 << 24) + 5
    maxd = int(np.floor(np.log2(cap)))
    t, o = SumTree(cap, dev), orc.Tree(cap)
    base = np.arange(0, cap, 97)
    w0 = rng.random(len(base))
    t.update(base, w0)
    o.update(base, w0)
    root = (1 << 11) - 1 + 300
    idx = np.concatenate([_subtree_ids(root, 11, cap, maxd, rng, 3000), rng.integers(0, 2047, 50),
                          _subtree_ids(root + 256, 11, cap, maxd, rng, 200)])
    rng.shuffle(idx)
    w = rng.random(len(idx))
    t.update(idx, w)
    o.update(idx, w)
    _assert_tree_equal(t, o)


# ---------------------------------------------------------------------- ApexDQN at size
def _tree_invariants(tree):
    """every node: sum == (val + sum[l]) + sum[r] in fp64 (the maintain order), and min is
    the reference's seeded min over the existing children (nodes ever maintained)"""
    s, m, v = _export(tree)
    cap = len(s)
    i = np.arange(cap)
    l, r = 2 * i + 1, 2 * i + 2
    sl = np.where(l < cap, s[np.minimum(l, cap - 1)], 0.0)
    sr = np.where(r < cap, s[np.minimum(r, cap - 1)], 0.0)
    want = (v + sl) + sr
    assert np.array_equal(s, want)
    ml = np.where(l < cap, m[np.minimum(l, cap - 1)], 0.0)
    mr = np.where(r < cap, m[np.minimum(r, cap - 1)], 0.0)
    mn = np.where(v != 0.0, v, 1.0)
    mn = np.where((ml != 0.0) & (ml < mn), ml, mn)
    mn = np.where((mr != 0.0) & (mr < mn), mr, mn)
    touched = s != 0.0
    assert np.array_equal(m[touched], mn[touched])
    return s, m, v


def _run_apex(dev, cfg, iters, prefill=0):
    from reth_amd.apex import ApexDQN

    ax = ApexDQN(cfg, device=dev)
    if prefill:
        ax.prefill(prefill)
    for _ in range(iters):
        ax.iteration()
    torch.cuda.synchronize()
    return ax


def _check_apex(ax, cfg, iters, prefill):
    size, tail, cnt, calls, steps = ax.replay.info()
    assert steps == ax.updates and ax.trainer.cur_step == ax.updates
    assert ax.env_steps == cfg.n_actors * iters
    emitted = cfg.n_actors * (iters - cfg.n_step - 1)  # fused actor: rows land one step later
    # cnt counts every sampler message's rows: appends and priority updates (sampler_loop.py)
    assert cnt == prefill + emitted + cfg.batch_size * ax.updates
    assert tail == (prefill + emitted) % cfg.capacity and size == min(prefill + emitted, cfg.capacity)
    assert ax.updates >= iters - 6 and calls == ax.updates + 1
    assert all(torch.isfinite(p).all() for p in ax.solver.q_network.parameters())
    act = ax.actors
    assert int(act.action.max()) < cfg.num_actions
    rows = act._sets[(act.pushes - 2) % 2]
    n = cfg.n_actors
    slots = (torch.arange(tail - n, tail, device=ax.device) + cfg.capacity) % cfg.capacity
    out = ax.replay.gather(slots)
    assert torch.equal(out[1], rows.a) and torch.equal(out[2], rows.r) and torch.equal(out[4], rows.done)
    assert torch.equal(out[0], act.frames[rows.s0]) and torch.equal(out[3], act.frames[rows.s1])


def _state(ax):
    s, m, v = _export(ax.replay.tree)
    size, tail = ax.replay.info()[:2]
    lo = max(0, tail - 4 * ax.cfg.n_actors)
    cols = ax.replay.gather(torch.arange(lo, tail, device=ax.device))
    small = [c.cpu() for c in (cols[1], cols[2], cols[4])]
    frames = [c.view(c.shape[0], -1).to(torch.int64).sum(1).cpu() for c in (cols[0], cols[3])]
    return [torch.from_numpy(x) for x in (s, m, v)] + small + frames, ax.replay.info()


def _collect():
    """free a dropped ApexDQN's HBM (its replay shard is hipMalloc'd by the library)"""
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("size", ["pong", "breakout"])
def test_apex_at_config_size(dev, size):
    """configs[1]: 256 actors, 1 M rows (prefilled), B = 512; configs[2]: 2,048 actors,
    A = 4, a 4 M-row shard (226 GB of row storage, filled by the actors).  Graph mode with
    learning on, then the counters / rows / tree checks, then graph == eager at lr = 0."""
    from reth_amd.apex import ApexConfig

    if size == "pong":
        kw = dict(n_actors=256, num_actions=6, capacity=1_000_000)
        prefill, iters = 1_000_000 - 256 * 10, 30
    else:
        kw = dict(n_actors=2048, num_actions=4, capacity=4_000_000)
        prefill, iters = 0, 30
    cfg = ApexConfig(batch_size=512, hip_graph=True, seed=3, **kw)
    ax = _run_apex(dev, cfg, iters, prefill)
    assert ax._graphs is not None and ax.actor_modes.get("dedup", 0) > 0
    _check_apex(ax, cfg, iters, prefill)
    _tree_invariants(ax.replay.tree)
    ax.close()
    ax = None
    _collect()
    # graph replay == eager (lr = 0 keeps the networks fixed), fewer iterations
    states = []
    for graph in (False, True):
        c = ApexConfig(batch_size=512, hip_graph=graph, seed=4, learning_rate=0.0, **kw)
        ax = _run_apex(dev, c, 14, prefill // 4)
        assert (ax._graphs is not None) == graph
        states.append(_state(ax))
        ax.close()
        ax = None
        _collect()
    (a, ia), (b, ib) = states
    assert ia == ib
    for x, y in zip(a, b):
        assert torch.equal(x, y)
