"""Actor-side kernels against the oracle: batched epsilon-greedy (explicit and Philox
draws), per-actor n-step adders (both numpy promotion modes, random done patterns), the
synthetic env's frame-stack invariants, and the vectorised actor loop's emitted rows."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_eps_greedy_explicit_and_philox(dev, orc):
    from reth_amd import _lib

    rng = np.random.default_rng(0)
    N, A = 1000, 6
    q = rng.standard_normal((N, A)).astype(np.float32)
    q[:50] = np.round(q[:50])  # ties
    q[50, 2] = np.nan
    eps = np.linspace(0.0, 1.0, N)
    u = rng.random(N)
    ra = rng.integers(0, A, N)
    qd, ed, ud, rd = (torch.as_tensor(x, device=dev) for x in (q, eps, u, ra))
    out = torch.empty(N, dtype=torch.int64, device=dev)
    _lib.call("rth_eps_greedy", qd.data_ptr(), N, A, 0, ed.data_ptr(), ud.data_ptr(), rd.data_ptr(), 0, 0, None,
              out.data_ptr(), _lib.stream_ptr())
    assert np.array_equal(out.cpu().numpy(), orc.eps_greedy(q, eps, u, ra))
    greedy = torch.argmax(torch.as_tensor(q), 1).numpy()
    sel = u >= eps
    assert np.array_equal(out.cpu().numpy()[sel], greedy[sel])  # torch.argmax first-max semantics
    # device RNG path: Philox(seed, counter, lane)
    seed, counter = 77, 5
    _lib.call("rth_eps_greedy", qd.data_ptr(), N, A, 0, ed.data_ptr(), None, None, seed, counter, None,
              out.data_ptr(), _lib.stream_ptr())
    pu = np.array([orc.philox_uniform(seed, counter, i, orc.STREAM_EXPLORE) for i in range(N)])
    pra = np.array([(int(orc.philox4x32([i, counter, 0, orc.STREAM_RANDACT], [seed, 0])[0]) * A) >> 32
                    for i in range(N)])
    assert np.array_equal(out.cpu().numpy(), orc.eps_greedy(q, eps, pu, pra))
    # the counter read from device memory (graph-replay form) gives the same draws
    cdev = torch.tensor([counter], dtype=torch.int64, device=dev)
    out2 = torch.empty_like(out)
    _lib.call("rth_eps_greedy", qd.data_ptr(), N, A, 0, ed.data_ptr(), None, None, seed, 999, cdev.data_ptr(),
              out2.data_ptr(), _lib.stream_ptr())
    assert torch.equal(out, out2)


def dueling_q(h):
    """Q = (V + adv) - mean(adv) from raw heads [n, A+1] in float32 (dqn_model.py:185-193);
    mean = sequential sum * (1/A) as torch's reduction computes it for short rows"""
    A = h.shape[1] - 1
    s = np.zeros(h.shape[0], np.float32)
    for j in range(A):
        s = (s + h[:, j]).astype(np.float32)
    mean = s * (np.float32(1.0) / np.float32(A))
    return (h[:, A:A + 1] + h[:, :A]) - mean[:, None]


def test_eps_greedy_dueling_heads(dev, orc):
    from reth_amd import _lib

    rng = np.random.default_rng(3)
    N, A = 2000, 6
    h = (rng.standard_normal((N, A + 1)) * 4).astype(np.float32)
    h[:100, :A] = np.round(h[:100, :A])  # ties survive the dueling combine
    eps = rng.random(N) * 0.2
    u, ra = rng.random(N), rng.integers(0, A, N)
    hd, ed, ud, rd = (torch.as_tensor(x, device=dev) for x in (h, eps, u, ra))
    out = torch.empty(N, dtype=torch.int64, device=dev)
    _lib.call("rth_eps_greedy", hd.data_ptr(), N, A, 1, ed.data_ptr(), ud.data_ptr(), rd.data_ptr(), 0, 0, None,
              out.data_ptr(), _lib.stream_ptr())
    assert np.array_equal(out.cpu().numpy(), orc.eps_greedy(dueling_q(h), eps, u, ra))


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("n_step", [1, 3, 5])
def test_nstep_device_vs_oracle(dev, orc, mode, n_step):
    from reth_amd import _lib

    N, T = 300, 40
    rng = np.random.default_rng(10 * n_step + mode)
    h = _lib.c_vp()
    _lib.call("rth_nstep_create", N, n_step, 0.99, mode, dev.index, _lib.ctypes.byref(h))
    oracles = [orc.NStep(n_step, 0.99, mode) for _ in range(N)]
    z = lambda dt: torch.zeros(N, dtype=dt, device=dev)
    emit, s0o, ao, s1o = z(torch.int32), z(torch.int64), z(torch.int64), z(torch.int64)
    ro, do = z(torch.float32), z(torch.float32)
    p_done = rng.choice([0.0, 0.05, 0.5], N)
    for t in range(T):
        s0 = np.arange(N) * 1000 + t
        a = rng.integers(0, 6, N)
        r = np.where(rng.random(N) < 0.5, rng.standard_normal(N), rng.choice([-1.0, 0.0, 1.0], N)).astype(np.float32)
        s1 = s0 + 500
        d = (rng.random(N) < p_done).astype(np.float32)
        dd = [torch.as_tensor(x, device=dev) for x in (s0, a, r, s1, d)]
        _lib.call("rth_nstep_push", h.value, *[x.data_ptr() for x in dd], emit.data_ptr(), s0o.data_ptr(), ao.data_ptr(),
                  ro.data_ptr(), s1o.data_ptr(), do.data_ptr(), _lib.stream_ptr())
        got = [x.cpu().numpy() for x in (emit, s0o, ao, ro, s1o, do)]
        for i in range(N):
            row = oracles[i].push(s0[i], a[i], r[i], s1[i], d[i])
            assert bool(got[0][i]) == (row is not None)
            if row is not None:
                assert (got[1][i], got[2][i], got[4][i]) == (row[0], row[1], row[3])
                assert got[3][i].tobytes() == np.float32(row[2]).tobytes()
                assert got[5][i] == row[4]
    _lib.lib().rth_nstep_destroy(h.value)


def test_synth_env_stack_invariants(dev):
    from reth_amd import _lib
    from reth_amd.actors import OBS_SHAPE

    N, ring = 64, 16
    frames = torch.zeros((N * ring, *OBS_SHAPE), dtype=torch.uint8, device=dev)
    cur = torch.zeros(N, dtype=torch.int64, device=dev)
    _lib.call("rth_synth_env_reset", frames.data_ptr(), N, ring, 5, cur.data_ptr(), _lib.stream_ptr())
    base = torch.arange(N, device=dev) * ring
    f0 = frames[base + 1]
    assert torch.equal(cur.cpu(), torch.ones(N, dtype=torch.int64))
    assert all(torch.equal(f0[:, k], f0[:, 0]) for k in range(4))  # reset: one frame x4
    z = lambda dt: torch.zeros(N, dtype=dt, device=dev)
    r, d, s0, s1 = z(torch.float32), z(torch.float32), z(torch.int64), z(torch.int64)
    dones = 0
    for t in range(1, 40):
        prev = frames[base + cur].clone()
        prev_cur = cur.clone()
        _lib.call("rth_synth_env_step", frames.data_ptr(), N, ring, t, None, cur.data_ptr(), None, 5, 0.5, 0.1,
                  r.data_ptr(), d.data_ptr(), s0.data_ptr(), s1.data_ptr(), _lib.stream_ptr())
        nxt = frames[s1]
        assert torch.equal(s0, base + prev_cur)
        assert torch.equal(nxt[:, :3], prev[:, 1:])  # FrameStack shift + one new frame
        assert set(r.cpu().numpy().tolist()) <= {-1.0, 0.0, 1.0}
        dn = d.bool()
        dones += int(dn.sum())
        assert torch.equal(cur[~dn], (s1 - base)[~dn])
        if dn.any():
            rs = frames[(base + cur)[dn]]
            assert all(torch.equal(rs[:, k], rs[:, 0]) for k in range(4))
    assert dones > 0
    # determinism: same seed -> same frames
    frames2 = torch.zeros_like(frames)
    cur2 = torch.zeros_like(cur)
    _lib.call("rth_synth_env_reset", frames2.data_ptr(), N, ring, 5, cur2.data_ptr(), _lib.stream_ptr())
    assert torch.equal(frames2[base + 1], f0)


def test_vec_actors_rows_follow_nstep_semantics(dev, orc):
    """emitted rows reference the right stacks and carry the oracle's n-step reward"""
    from reth_amd.actors import VecActors
    from reth_amd.model import DQNNetwork

    torch.manual_seed(0)
    N = 32
    net = DQNNetwork((4, 84, 84), 6).to(dev)
    act = VecActors(N, 6, n_step=3, gamma=0.99, device=dev, seed=3, p_reward=0.3, p_done=0.2, nstep_mode=0)
    oracles = [orc.NStep(3, 0.99, 0) for _ in range(N)]
    for t in range(12):
        warm = act.step(net)
        s0h, s1h = act.s0_h.cpu().numpy(), act.s1_h.cpu().numpy()
        a, r, d = act.action.cpu().numpy(), act.reward.cpu().numpy(), act.done.cpu().numpy()
        rows = [oracles[i].push(s0h[i], a[i], r[i], s1h[i], d[i]) for i in range(N)]
        assert warm == (rows[0] is not None) and all((x is None) == (rows[0] is None) for x in rows)
        if warm:
            got = [x.cpu().numpy() for x in (act.row_s0, act.row_a, act.row_r, act.row_s1, act.row_done)]
            for i in range(N):
                assert (got[0][i], got[1][i], got[3][i]) == (rows[i][0], rows[i][1], rows[i][3])
                assert got[2][i] == rows[i][2] and got[4][i] == rows[i][4]
            td = act.prioritise(net)
            # calc_loss on the actor copy: target == online (dqn_solver.py:133-137)
            s0f = act.frames[act.row_s0].float()
            s1f = act.frames[act.row_s1].float()
            with torch.no_grad():
                q0, q1 = net(s0f), net(s1f)
            want = orc.td_error(q0.cpu().numpy(), q1.cpu().numpy(), q1.cpu().numpy(), got[1], got[2], got[4],
                                np.float32(0.99 ** 3))
            np.testing.assert_allclose(td.cpu().numpy(), np.abs(want), rtol=1e-5, atol=1e-5)


def test_step_fused_matches_step_then_prioritise(dev):
    """the fused actor step (act + the previous rows' calc_loss in one 3N forward) emits the
    same rows and the same |td| (one step later) as step() + prioritise()"""
    from reth_amd.actors import VecActors
    from reth_amd.model import DQNNetwork

    torch.manual_seed(0)
    N = 24
    net = DQNNetwork((4, 84, 84), 6).to(dev, memory_format=torch.channels_last)
    net.hwc_features = True
    kw = dict(n_step=3, gamma=0.99, device=dev, seed=9, p_reward=0.3, p_done=0.1, channels_last=True)
    a, b = VecActors(N, 6, **kw), VecActors(N, 6, **kw)
    want = []
    for t in range(10):
        if a.step(net):
            want.append((a.row_s0.clone(), a.row_a.clone(), a.row_r.clone(), a.row_done.clone(), a.prioritise(net)))
        td, rows = b.step_fused(net)
        assert torch.equal(a.action, b.action)
        assert torch.equal(a.frames[a.current_obs_handles()], b.frames[b.current_obs_handles()])
        if td is not None:
            s0, ra, rr, rd, wtd = want[-2]
            assert torch.equal(rows.s0, s0) and torch.equal(rows.a, ra) and torch.equal(rows.r, rr)
            assert torch.equal(rows.done, rd)
            torch.testing.assert_close(td, wtd, rtol=1e-5, atol=1e-5)  # batch 3N vs 2N GEMM blocking


def test_step_fused_dedup_matches_full(dev):
    """dedup mode (forward over the acting + terminal stacks only, rows' heads from the
    per-stack cache) gives the actions and |td| of the full 3-way forward, through many
    episode ends (p_done = 0.25) and a weights change (the cache is rebuilt: full mode for
    n + 2 steps)"""
    from reth_amd.actors import VecActors
    from reth_amd.model import DQNNetwork

    torch.manual_seed(1)
    N = 40
    net = DQNNetwork((4, 84, 84), 6).to(dev, memory_format=torch.channels_last)
    net.hwc_features = True
    net.requires_grad_(False)
    kw = dict(n_step=3, gamma=0.99, device=dev, seed=21, p_reward=0.3, p_done=0.25, channels_last=True)
    a, b = VecActors(N, 6, **kw), VecActors(N, 6, **kw)
    modes = []
    for t in range(24):
        if t == 12:  # actor weights reload
            with torch.no_grad():
                for p in net.parameters():
                    p.add_(torch.randn_like(p) * 1e-3)
            a.weights_changed()
            b.weights_changed()
        dedup = b.dedup_ready(net)
        modes.append(dedup)
        ta, ra = a.step_fused(net, dedup=False)
        tb, rb = b.step_fused(net)
        assert torch.equal(a.action, b.action), t
        assert torch.equal(a.n_ext, b.n_ext)
        if ta is not None:
            assert torch.equal(ra.s0, rb.s0) and torch.equal(ra.s1, rb.s1) and torch.equal(ra.done, rb.done)
            torch.testing.assert_close(tb, ta, rtol=1e-5, atol=1e-5)
    assert modes[:5] == [False] * 5 and all(modes[5:12]) and modes[12:17] == [False] * 5 and all(modes[17:])
    assert int(b.n_ext) > N or bool(b.done.any())  # the episodes did end


def test_compact_flagged(dev):
    from reth_amd._lib import call, ptr, stream_ptr

    g = torch.Generator(device=dev).manual_seed(4)
    for n, cap in [(0, 5), (1, 1), (37, 37), (256, 256), (257, 300), (2048, 2048), (3000, 100)]:
        flag = (torch.rand(max(n, 1), device=dev, generator=g) < 0.3).float()[:n]
        vals = torch.randint(0, 1 << 40, (n,), device=dev, generator=g)
        out = torch.empty(cap, dtype=torch.int64, device=dev)
        cnt = torch.empty(1, dtype=torch.int64, device=dev)
        call("rth_compact_flagged", ptr(flag), ptr(vals), n, ptr(out), cap, -7, 100, ptr(cnt), stream_ptr())
        want = vals[flag != 0][:cap]
        k = want.numel()
        assert int(cnt) == 100 + k
        assert torch.equal(out[:k], want) and bool((out[k:] == -7).all())
