"""Device sum-tree / PER parity: bit-exact against the reference's golden vectors and the
oracle (tree state, find, sample indices), IS weights within fp64 rounding."""
import hashlib

import numpy as np
import pytest
import torch

from test_oracle_golden import SMALL_TAGS, large_inputs

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


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def export(t):
    s, m, v = t.export()
    torch.cuda.synchronize()
    return s.cpu().numpy(), m.cpu().numpy(), v.cpu().numpy()


@pytest.mark.parametrize("tag", SMALL_TAGS)
def test_golden_small(golden, dev, tag):
    from reth_amd.replay import SumTree

    g = golden("sumtree_small.npz")
    t = SumTree(int(g[f"{tag}/capacity"]), dev)
    for k in range(int(g[f"{tag}/n_upd"])):
        t.update(g[f"{tag}/upd{k}_idx"], g[f"{tag}/upd{k}_w"])
    s, m, v = export(t)
    assert np.array_equal(s, g[f"{tag}/sum"])
    assert np.array_equal(m, g[f"{tag}/min"])
    assert np.array_equal(v, g[f"{tag}/val"])
    assert t.min() == float(g[f"{tag}/tree_min"])
    idx, val = t.find(g[f"{tag}/targets"])
    assert np.array_equal(idx.cpu().numpy(), g[f"{tag}/find"])
    idx, val = t.sample(len(g[f"{tag}/sample_u"]), uniforms=g[f"{tag}/sample_u"])
    assert np.array_equal(idx.cpu().numpy(), g[f"{tag}/sample_idx"])
    assert np.array_equal(val.cpu().numpy(), g[f"{tag}/sample_val"])


def test_golden_large_pong_depth(golden, dev):
    """C = 2^20 (21 levels): FIFO-range appends through the fused PER update (f32 |td|,
    alpha 0.5) and 40 learner updates; state hashes equal the reference's."""
    from reth_amd.replay import PERSampler

    g = golden("sumtree_large.npz")
    cap, chunk = int(g["capacity"]), int(g["chunk"])
    fills, learn = large_inputs(g)
    per = PERSampler(cap, alpha=0.5, beta=0.4, device=dev)
    allfill = torch.as_tensor(np.concatenate(fills), device=dev)
    for k in range(len(fills)):
        per.update(torch.arange(k * chunk, (k + 1) * chunk, device=dev), allfill[k * chunk:(k + 1) * chunk])
    for idx, td in learn:
        per.update(idx, td)
    s, m, v = export(per.sumtree)
    assert sha(s) == str(g["sha_sum"]) and sha(m) == str(g["sha_min"]) and sha(v) == str(g["sha_val"])
    idx, val = per.sumtree.sample(int(g["batch"]), uniforms=g["sample_u"])
    assert np.array_equal(idx.cpu().numpy(), g["sample_idx"])
    assert np.array_equal(val.cpu().numpy(), g["sample_val"])


def test_one_shot_bulk_update_matches_sequential(golden, dev, orc):
    """the whole 2^20 fill as ONE update call (256 LDS chunks in order) == sequential"""
    from reth_amd.replay import SumTree

    rng = np.random.default_rng(11)
    cap = 1 << 16
    w = rng.random(cap + 5000)
    idx = np.concatenate([np.arange(cap), rng.integers(0, cap, 5000)])
    t = SumTree(cap, dev)
    t.update(idx, w)
    o = orc.Tree(cap)
    o.update(idx, w)
    s, m, v = export(t)
    assert np.array_equal(s, o.sum) and np.array_equal(m, o.min_) and np.array_equal(v, o.val)


@pytest.mark.parametrize("seed", range(12))
def test_random_against_oracle(dev, orc, seed):
    """random capacities (ragged last level), duplicates, zeros, never-filled slots,
    batches crossing the 4096-key LDS chunk, and out-of-order indices"""
    from reth_amd.replay import SumTree

    rng = np.random.default_rng(1000 + seed)
    cap = int(rng.choice([1, 2, 3, 7, 64, 100, 1023, 1024, 1025, 5000, 70000]))
    t = SumTree(cap, dev)
    o = orc.Tree(cap)
    for _ in range(4):
        n = int(rng.choice([1, 5, 63, 512, 4096, 4097, 9000]))
        hi = max(1, int(cap * rng.choice([0.3, 1.0])))
        idx = rng.integers(0, hi, n)
        if n > 8:
            idx[: n // 4] = idx[n // 4: 2 * (n // 4)]  # forced duplicates
        w = rng.random(n)
        w[rng.random(n) < 0.05] = 0.0
        t.update(idx, w)
        o.update(idx, w)
    s, m, v = export(t)
    assert np.array_equal(v, o.val)
    assert np.array_equal(s, o.sum)
    assert np.array_equal(m, o.min_)
    u = rng.random(257)
    gi, gv = t.sample(257, uniforms=u)
    oi, ov = o.sample(u)
    assert np.array_equal(gi.cpu().numpy(), oi) and np.array_equal(gv.cpu().numpy(), ov)
    tg = np.concatenate([rng.random(100) * o.total() * 1.1, [0.0, o.total(), o.total() + 1e-6]])
    fi, _ = t.find(tg)
    assert np.array_equal(fi.cpu().numpy(), np.array([o.find(x) for x in tg]))


def test_clear_and_import(dev, orc):
    from reth_amd.replay import SumTree

    t = SumTree(777, dev)
    t.update(np.arange(777), np.ones(777))
    t.clear()
    s, m, v = export(t)
    assert not s.any() and not m.any() and not v.any() and t.min() == 1.0
    o = orc.Tree(777)
    o.update(np.arange(300), np.random.default_rng(0).random(300))
    t.load(o.sum, o.min_, o.val)
    u = np.random.default_rng(1).random(64)
    assert np.array_equal(t.sample(64, uniforms=u)[0].cpu().numpy(), o.sample(u)[0])


@pytest.mark.parametrize("tag,alpha", [("a05", 0.5), ("a06", 0.6)])
def test_per_sampler_golden_sequence(golden, dev, tag, alpha):
    from reth_amd.replay import PERSampler

    g = golden("per.npz")
    w = g[f"{tag}/w"]
    per = PERSampler(2000, alpha=alpha, beta="0.4,1,2000000", device=dev)
    for st in range(0, 1500, 64):
        n = min(64, 1500 - st)
        per.update(np.arange(st, st + n, dtype=np.int32), w[st:st + n])
    for k in range(8):
        idx, isw = per.sample(64, uniforms=g[f"{tag}/s{k}_u"])
        assert np.array_equal(idx.cpu().numpy(), g[f"{tag}/s{k}_idx"])
        np.testing.assert_allclose(isw.cpu().numpy(), g[f"{tag}/s{k}_isw"], rtol=1e-6 if alpha != 0.5 else 1e-13)
        per.on_step()
        per.update(idx, w[1500 + 64 * k: 1564 + 64 * k])
    s, _, v = export(per.sumtree)
    if alpha == 0.5:
        assert sha(s) == str(g[f"{tag}/final_sha_sum"]) and sha(v) == str(g[f"{tag}/final_sha_val"])


def test_per_normalize_kernel(dev, orc):
    from reth_amd import _lib

    rng = np.random.default_rng(3)
    w = (rng.random(100000) * 5).astype(np.float32)
    w[:4] = [0.0, 1e-30, 1e30, 3.0]
    for alpha in (0.5, 0.6, 1.0, 0.7):
        src = torch.as_tensor(w, device=dev)
        out = torch.empty_like(src)
        _lib.call("rth_per_normalize", src.data_ptr(), src.numel(), alpha, out.data_ptr(), _lib.stream_ptr())
        assert np.array_equal(out.cpu().numpy(), orc.per_normalize(w, alpha)), alpha


def test_device_rng_sampling_matches_oracle_philox(dev, orc):
    """without explicit uniforms the device draws Philox(seed, counter, lane): same
    uniforms as the oracle's restatement -> same indices"""
    from reth_amd.replay import SumTree

    rng = np.random.default_rng(9)
    cap = 50000
    w = rng.random(cap)
    t = SumTree(cap, dev)
    t.update(np.arange(cap), w)
    o = orc.Tree(cap)
    o.update(np.arange(cap), w)
    for counter in (0, 1, 2 ** 33 + 5):
        idx, _ = t.sample(512, seed=1234, counter=counter)
        u = np.array([orc.philox_uniform(1234, counter, i, orc.STREAM_SAMPLE) for i in range(512)])
        assert np.array_equal(idx.cpu().numpy(), o.sample(u)[0])


def test_per_distribution(dev):
    """reth/test/test_buffer.py:135-167: sampled frequencies track p^alpha (L1 < 0.1),
    before and after update_priorities"""
    from reth_amd.replay import PERSampler

    cap = 100
    per = PERSampler(cap, alpha=0.6, beta=0.4, device=dev, seed=5)
    rng = np.random.default_rng(0)

    def check(weights):
        cnt = np.zeros(cap)
        for _ in range(100):
            idx, _ = per.sample(64)
            np.add.at(cnt, idx.cpu().numpy(), 1)
        p = (weights + 1e-6) ** 0.6
        a, b = cnt / cnt.sum(), p / p.sum()
        assert (np.abs(a - b) / b).sum() / cap < 0.1

    w = rng.random(cap).astype(np.float32)
    per.update(np.arange(cap), w)
    check(w)
    w = rng.random(cap).astype(np.float32)
    per.update(np.arange(cap), w)
    check(w)


def test_find_and_sample_ragged(dev, orc, golden):
    """rth_sumtree_find (lane groups of 2^4 lanes, 4 levels per round trip) and the sampler
    (k_tree_sample_deep: 10 levels staged in LDS, 2 per round trip below) return the oracle's
    indices: ragged trees, zeros, targets at and past the total, the golden small trees"""
    from reth_amd.replay import SumTree

    rng = np.random.default_rng(77)
    for cap in (1, 2, 3, 7, 31, 33, 1000, 65537, 300000):
        t = SumTree(cap, dev)
        o = orc.Tree(cap)
        idx = rng.integers(0, cap, max(1, cap // 2))
        w = rng.random(len(idx))
        w[rng.random(len(idx)) < 0.1] = 0.0
        t.update(idx, w)
        o.update(idx, w)
        u = rng.random(300)  # not a multiple of any group or workgroup size
        gi, gv = t.sample(300, uniforms=u)
        oi, ov = o.sample(u)
        assert np.array_equal(gi.cpu().numpy(), oi) and np.array_equal(gv.cpu().numpy(), ov), cap
        tg = np.concatenate([rng.random(61) * o.total() * 1.05, [0.0, o.total(), o.total() + 1e-6]])
        fi, _ = t.find(tg)
        assert np.array_equal(fi.cpu().numpy(), np.array([o.find(x) for x in tg])), cap
    g = golden("sumtree_small.npz")
    for tag in SMALL_TAGS:
        t = SumTree(int(g[f"{tag}/capacity"]), dev)
        for k in range(int(g[f"{tag}/n_upd"])):
            t.update(g[f"{tag}/upd{k}_idx"], g[f"{tag}/upd{k}_w"])
        idx, _ = t.find(g[f"{tag}/targets"])
        assert np.array_equal(idx.cpu().numpy(), g[f"{tag}/find"]), tag
        idx, val = t.sample(len(g[f"{tag}/sample_u"]), uniforms=g[f"{tag}/sample_u"])
        assert np.array_equal(idx.cpu().numpy(), g[f"{tag}/sample_idx"]), tag
