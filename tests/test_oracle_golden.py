"""Pin the CPU oracle (oracle/reth_oracle.c) against golden vectors generated from the
reference itself (tests/golden/make_golden.py).  CPU only."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

SMALL_TAGS = ["c10", "c5", "c1", "c1000", "c3000", "c4097"]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("tag", SMALL_TAGS)
def test_sumtree_small_update_find_sample(golden, orc, tag):
    g = golden("sumtree_small.npz")
    t = orc.Tree(int(g[f"{tag}/capacity"]))
    for k in range(int(g[f"{tag}/n_upd"])):
        t.update(g[f"{tag}/upd{k}_idx"], g[f"{tag}/upd{k}_w"])
    # bit-exact state, including the min() quirk of never-touched children
    assert np.array_equal(t.sum, g[f"{tag}/sum"])
    assert np.array_equal(t.min_, g[f"{tag}/min"])
    assert np.array_equal(t.val, g[f"{tag}/val"])
    assert t.min() == float(g[f"{tag}/tree_min"])
    found = np.array([t.find(x) for x in g[f"{tag}/targets"]])
    assert np.array_equal(found, g[f"{tag}/find"])
    idx, val = t.sample(g[f"{tag}/sample_u"])
    assert np.array_equal(idx, g[f"{tag}/sample_idx"])
    assert np.array_equal(val, g[f"{tag}/sample_val"])


def test_inorder_mass_mapping(orc):
    """capacity 10, equal priorities -> [7,3,8,1,9,4,0,5,2,6]"""
    t = orc.Tree(10)
    t.update(np.arange(10), np.ones(10))
    assert [t.find(k + 0.5) for k in range(10)] == [7, 3, 8, 1, 9, 4, 0, 5, 2, 6]


def large_inputs(g):
    """regenerate the large-tree inputs exactly as make_golden.gen_sumtree_large drew them"""
    rng = np.random.default_rng(int(g["seed"]))
    cap, chunk = int(g["capacity"]), int(g["chunk"])
    fills = [rng.random(chunk, dtype=np.float32) for _ in range(0, cap, chunk)]
    learn = []
    for _ in range(int(g["n_learn"])):
        idx = rng.integers(0, cap, int(g["batch"]))
        learn.append((idx, rng.random(int(g["batch"]), dtype=np.float32) * np.float32(3.0)))
    return fills, learn


def test_sumtree_large_pong_depth(golden, orc):
    g = golden("sumtree_large.npz")
    cap, chunk = int(g["capacity"]), int(g["chunk"])
    fills, learn = large_inputs(g)
    t = orc.Tree(cap)
    for k, td in enumerate(fills):
        t.update(np.arange(k * chunk, (k + 1) * chunk), orc.per_normalize(td, 0.5).astype(np.float64))
    for idx, td in learn:
        t.update(idx, orc.per_normalize(td, 0.5).astype(np.float64))
    assert sha(t.sum) == str(g["sha_sum"])
    assert sha(t.min_) == str(g["sha_min"])
    assert sha(t.val) == str(g["sha_val"])
    idx, val = t.sample(g["sample_u"])
    assert np.array_equal(idx, g["sample_idx"]) and np.array_equal(val, g["sample_val"])


@pytest.mark.parametrize("tag,alpha", [("a05", 0.5), ("a06", 0.6)])
def test_per_normalize(golden, orc, tag, alpha):
    g = golden("per.npz")
    ours = orc.per_normalize(g[f"{tag}/w"], alpha)
    ref = g[f"{tag}/norm"]
    assert ours.dtype == np.float32 and ref.dtype == np.float32
    if alpha == 0.5:  # numpy's `** 0.5` is sqrt: correctly rounded everywhere -> exact
        assert np.array_equal(ours, ref)
    else:  # numpy's f32 pow is platform-dependent (SVML here); ours is correctly rounded
        ulps = np.abs(ours.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
        assert ulps.max() <= 1


@pytest.mark.parametrize("tag,alpha", [("a05", 0.5), ("a06", 0.6)])
def test_per_sampler_sequence(golden, orc, tag, alpha):
    """append in 64-row messages, then 8 x (sample, on_step, update) like sampler_loop"""
    from reth_amd.schedule import Schedule

    g = golden("per.npz")
    w = g[f"{tag}/w"]
    t = orc.Tree(2000)
    for st in range(0, 1500, 64):
        n = min(64, 1500 - st)
        t.update(np.arange(st, st + n), orc.per_normalize(w[st:st + n], alpha).astype(np.float64))
    beta = Schedule.from_str("0.4,1,2000000")
    for k in range(8):
        assert beta.value() == g[f"{tag}/betas"][k]
        idx, p = t.sample(g[f"{tag}/s{k}_u"])
        isw = orc.per_is_weights(p, t.min(), beta.value())
        assert np.array_equal(idx, g[f"{tag}/s{k}_idx"])
        np.testing.assert_allclose(isw, g[f"{tag}/s{k}_isw"], rtol=1e-6 if alpha != 0.5 else 1e-13)
        beta.step()
        t.update(idx, orc.per_normalize(w[1500 + 64 * k: 1564 + 64 * k], alpha).astype(np.float64))
    if alpha == 0.5:
        assert sha(t.sum) == str(g[f"{tag}/final_sha_sum"])
        assert sha(t.val) == str(g[f"{tag}/final_sha_val"])
    assert t.total() == pytest.approx(float(g[f"{tag}/final_sum"]), rel=1e-12 if alpha == 0.5 else 1e-6)


def test_schedule_and_fifo(orc):
    from reth_amd.schedule import Interval, Schedule

    with open(os.path.join(GOLDEN, "schedule_fifo.json")) as f:
        ref = json.load(f)
    for case in ref["cases"]:
        s = Schedule.from_str(case["spec"])
        assert [float(s.value(k)).hex() for k in ref["steps"]] == case["value"]
        assert [float(s.step()).hex() for _ in range(5)] == case["step_seq"]
        if isinstance(case["spec"], str):
            parts = case["spec"].split(",")
            method = parts[0] if len(parts) == 4 else "linear"
            lo, hi, n = float(parts[-3]), float(parts[-2]), int(parts[-1])
            got = [float(orc.schedule_value(method, lo, hi, n, k)).hex() for k in ref["steps"]]
            assert got == case["value"]
    for bad in ref["invalid"]:
        if bad["raises"]:
            with pytest.raises(Exception):
                Schedule.from_str(bad["spec"])
    tail = 0
    for n, want in zip(ref["fifo_requests"], ref["fifo_indices"]):
        got, tail = orc.fifo_indices(ref["fifo_capacity"], tail, n)
        assert got.tolist() == want
    calls = []
    iv = Interval(lambda: calls.append(1), 3)
    for _ in range(10):
        iv()
    assert len(calls) == 3


def test_nstep_streams_nep50(golden, orc):
    """the reference NStepAdder ran under numpy 2 here (NEP 50): oracle mode 1 is bit-exact"""
    g = golden("nstep.npz")
    tags = sorted({k.rsplit("/", 1)[0] for k in g.keys() if k.count("/") == 2})
    assert tags
    for tag in tags:
        n = int(tag.split("/")[0][1:])
        ad = orc.NStep(n, 0.99, mode=1)
        rows = []
        for t, (a, r, d) in enumerate(zip(g[f"{tag}/actions"], g[f"{tag}/rewards"], g[f"{tag}/dones"])):
            row = ad.push(t, a, r, t, d)
            if row is not None:
                rows.append((t,) + row)
        assert len(rows) == len(g[f"{tag}/emit_t"]), tag
        for k, (t, s0, a, r, s1, d) in enumerate(rows):
            assert t == g[f"{tag}/emit_t"][k] and s0 == g[f"{tag}/emit_s0"][k] and a == g[f"{tag}/emit_a"][k]
            assert s1 == g[f"{tag}/emit_s1"][k] and d == g[f"{tag}/emit_done"][k]
            assert np.float32(r).tobytes() == g[f"{tag}/emit_r"][k].tobytes(), (tag, k)


def test_nstep_terminal_quirk_legacy(orc):
    """rewards 1, done at the 3rd push; older rows keep done=0 and bootstrap
    from the terminal s1 (numpy-1.19 promotion, mode 0)"""
    ad = orc.NStep(3, 0.99, mode=0)
    out = [ad.push(t, 0, 1.0, t + 1, 1.0 if t == 2 else 0.0) for t in range(6)]
    rows = [r for r in out if r is not None]
    assert rows[0][0] == 0 and rows[0][3] == 3 and rows[0][4] == 0.0
    assert rows[0][2] == np.float32(np.float64(np.float32(1.0) + 0.99) + 0.99 * 0.99)
    assert rows[1][2] == np.float32(1.99) and rows[1][3] == 3 and rows[1][4] == 0.0
    assert rows[2][2] == np.float32(1.0) and rows[2][4] == 1.0


@pytest.mark.parametrize("name", ["dqn_pong_b8.npz", "dqn_pong_b32.npz"])
def test_td_error_restatement(golden, orc, name):
    """the oracle's TD restatement reproduces the reference's torch-CPU td bit for bit"""
    g = golden(name)
    td = orc.td_error(g["q_s0"], g["q_s1_online"], g["q_s1_target"], g["a"], g["r"], g["done"],
                      np.float32(0.99 ** 3))
    assert np.array_equal(td, g["td"])
    assert np.array_equal(np.abs(td), g["calc_loss"])


def test_td_huber_gradient_matches_torch(orc):
    """dq from the restatement == torch autograd of the reference's loss expression"""
    import torch
    import torch.nn.functional as F

    rng = np.random.default_rng(5)
    B, A = 64, 6
    td = (rng.standard_normal(B) * 2).astype(np.float32)
    td[:4] = [1.0, -1.0, 0.0, 1e-8]
    w = rng.random(B).astype(np.float32) + 0.1
    a = rng.integers(0, A, B)
    q = torch.zeros(B, A, requires_grad=True)
    onehot = F.one_hot(torch.as_tensor(a), A).float()
    tdt = torch.sum(q * onehot, 1) + torch.as_tensor(td)
    loss = F.smooth_l1_loss(tdt, torch.zeros_like(tdt), reduction="none")
    loss = (loss * torch.as_tensor(w)).mean()
    loss.backward()
    l, le, dq = orc.td_huber(td, w, a, A)
    assert np.array_equal(dq, q.grad.numpy())
    assert abs(float(l) - float(loss)) <= 1e-6 * max(1.0, abs(float(loss)))


def test_eps_greedy_and_argmax(orc):
    q = np.array([[1, 3, 3, 0], [np.nan, 1, np.nan, 2], [0, 0, 0, 0], [-1, -2, 5, 5]], np.float32)
    assert [orc.lib().orc_argmax_first(orc.P(np.ascontiguousarray(r)), 4) for r in q] == [1, 0, 0, 2]
    import torch

    assert torch.argmax(torch.as_tensor(q), 1).tolist() == [1, 0, 0, 2]
    out = orc.eps_greedy(q, [0.5] * 4, [0.1, 0.9, 0.5, 0.49], [7, 7, 7, 7])
    assert out.tolist() == [7, 0, 0, 7]


def test_philox_known_answer(orc):
    """Random123 known-answer vectors for philox4x32-10"""
    assert orc.philox4x32([0, 0, 0, 0], [0, 0]).tolist() == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert orc.philox4x32([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2).tolist() == [0x408F276D, 0x41C83B0E, 0xA20BC7C6,
                                                                          0x6D5451FD]
    assert orc.philox4x32([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0]).tolist() == [
        0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


# ---------------------------------------------------------------------------------------
# samplers / in-process buffers: the oracle restatements against the reference's outputs
# (tests/golden/buffers.npz, generated from the reference modules by make_golden.py)
# ---------------------------------------------------------------------------------------
def _ops(g, key):
    return [(str(x)[0], int(str(x)[1:])) for x in g[key]]


def test_fifo_sampler_restatement(golden, orc):
    g = golden("buffers.npz")
    s = orc.FIFOSampler(50)
    for k, (op, n) in enumerate(_ops(g, "fifo_ops")):
        if op == "s":
            assert s.ready_sample(n) == bool(g[f"fifo{k}_ready"])
            i, w = s.sample(n)
            assert np.array_equal(i, g[f"fifo{k}_idx"]) and np.array_equal(w, g[f"fifo{k}_w"])
        else:
            s.update(g[f"fifo{k}_in_idx"], g[f"fifo{k}_in_w"])


def uniforms_for_positions(pos, tail):
    """u with floor(u * tail) == pos (the reference drew positions with choice(tail, B))"""
    return (np.asarray(pos, np.float64) + 0.5) / tail


def test_uniform_sampler_restatement(golden, orc):
    g = golden("buffers.npz")
    s = orc.UniformSampler(64)
    for k, (op, n) in enumerate(_ops(g, "uni_ops")):
        if op == "s":
            assert s.tail == int(g[f"uni{k}_tail"])
            i, w = s.sample(uniforms_for_positions(g[f"uni{k}_pos"], s.tail))
            assert np.array_equal(i, g[f"uni{k}_idx"]) and np.array_equal(w, g[f"uni{k}_w"])
            assert w.dtype == np.int64
        else:
            s.update(g[f"uni{k}_in_idx"])


def test_numpy_buffer_indices_restatement(golden, orc):
    g = golden("buffers.npz")
    tail, size = -1, 0
    for k in range(int(g["nb_steps"])):
        n = len(g[f"nb{k}_in0"])
        idx, tail, size = orc.numpy_buffer_indices(10, tail, size, n)
        assert np.array_equal(idx, g[f"nb{k}_ret"]) and tail == int(g[f"nb{k}_tail"]) and size == int(g[f"nb{k}_size"])


def test_prioritized_buffer_restatement(golden, orc):
    g = golden("buffers.npz")
    pb = orc.PrioritizedBuffer(100, 0.6, "0.4,1,1000")
    for k, op in enumerate(str(x) for x in g["pb_ops"]):
        if op == "batch_w":
            pb.append_batch(len(g[f"pb{k}_w"]), g[f"pb{k}_w"])
        elif op == "batch":
            pb.append_batch(len(g[f"pb{k}_d1"]))
        elif op == "update":
            pb.update_priorities(g[f"pb{k}_idx"], g[f"pb{k}_w"])
        else:
            idx, w = pb.sample(g[f"pb{k}_u"])
            assert np.array_equal(idx, g[f"pb{k}_idx"])
            np.testing.assert_allclose(w, g[f"pb{k}_isw"], rtol=1e-12, atol=0)
        assert np.array_equal(pb.tree.sum, g[f"pb{k}_sum"])


def test_oracle_gray_known_values(orc):
    """cv2 RGB2GRAY fixed point on the primaries (OpenCV gives 76 / 150 / 29) and area
    weights summing to one per output pixel"""
    px = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [0, 0, 0]]], np.uint8)
    assert orc.rgb2gray(px).tolist() == [[76, 150, 29, 255, 0]]  # OpenCV's RGB2GRAY values
    for tab in (orc.area_tab(160, 84, 1 / (84 / 160)), orc.area_tab(210, 84, 1 / (84 / 210))):
        assert all(abs(sum(float(w) for _, w in t) - 1) < 1e-6 for t in tab)
