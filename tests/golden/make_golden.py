"""Generate the golden vectors under tests/golden/ from the reference itself.

Run ONCE in the build container (where /root/reference exists):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It loads the reference's own Python modules (read-only, no bytecode written) with the
import shims described in SURVEY.md Appendix B (numba.njit -> identity, a minimal
gym.spaces, namespace packages that skip reth/__init__.py), runs them on seeded inputs
and writes inputs + outputs as small .npz/.json fixtures.  Nothing here is imported by
the product, by the GPU tests or by bench.py: only the committed fixtures travel.

Reference functions exercised (paths relative to /root/reference):
  reth_buffer/reth_buffer/utils/sumtree.py:5-113      NumbaSumTree, _numba_*  (live PER tree)
  reth_buffer/reth_buffer/sampler/per_sampler.py:5-35 PERSampler
  reth_buffer/reth_buffer/utils/schedule.py:4-52      Schedule
  reth_buffer/reth_buffer/cache_policy/fifo_policy.py FIFOPolicy
  reth/reth/utils/nstep_adder.py:5-28                 NStepAdder
  reth/reth/algorithm/dqn/dqn_solver.py:14-143        DQNSolver (calc_loss / update / act)
  reth/reth/algorithm/dqn/dqn_model.py:6-99           DQNNetwork / MLP_DQNNetwork

numba's JIT is replaced by plain Python: njit without fastmath is IEEE with the same
operation order, so the deterministic arithmetic is identical; numba's private RNG stream
is not reproduced, so every sample fixture records its uniforms explicitly.
"""
import hashlib
import importlib.util
import json
import os
import sys
import types

sys.dont_write_bytecode = True

import numpy as np

REF = os.environ.get("RETH_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------- shims
def _install_shims():
    numba = types.ModuleType("numba")
    numba.njit = lambda f=None, **kw: (f if f is not None else (lambda g: g))
    sys.modules["numba"] = numba

    gym = types.ModuleType("gym")
    spaces = types.ModuleType("gym.spaces")

    class Discrete:
        def __init__(self, n):
            self.n = n

    class Box:
        def __init__(self, low, high, shape, dtype=None):
            self.low, self.high, self.shape = low, high, tuple(shape)

    spaces.Discrete, spaces.Box = Discrete, Box
    gym.spaces = spaces
    gym.Env = object
    sys.modules["gym"] = gym
    sys.modules["gym.spaces"] = spaces


def _pkg(name):
    m = types.ModuleType(name)
    m.__path__ = []
    sys.modules[name] = m
    return m


def _load(modname, relpath):
    spec = importlib.util.spec_from_file_location(modname, os.path.join(REF, relpath))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[modname] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference():
    _install_shims()
    R = types.SimpleNamespace()
    # reth_buffer live tree + PER sampler + schedule + FIFO
    _pkg("rb")
    rbu = _pkg("rb.utils")
    R.sumtree = _load("rb.utils.sumtree", "reth_buffer/reth_buffer/utils/sumtree.py")
    R.schedule = _load("rb.utils.schedule", "reth_buffer/reth_buffer/utils/schedule.py")
    rbu.NumbaSumTree = R.sumtree.NumbaSumTree
    rbu.Schedule = R.schedule.Schedule
    _pkg("rb.sampler")
    _load("rb.sampler.base_sampler", "reth_buffer/reth_buffer/sampler/base_sampler.py")
    R.per = _load("rb.sampler.per_sampler", "reth_buffer/reth_buffer/sampler/per_sampler.py")
    _pkg("rb.cache_policy")
    _load("rb.cache_policy.base_policy", "reth_buffer/reth_buffer/cache_policy/base_policy.py")
    R.fifo = _load("rb.cache_policy.fifo_policy", "reth_buffer/reth_buffer/cache_policy/fifo_policy.py")
    # reth: utils + dqn (skip reth/__init__.py, which imports env -> gym/cv2)
    _pkg("reth")
    _pkg("reth.utils").__path__ = [os.path.join(REF, "reth/reth/utils")]
    R.rutils = _load("reth.utils", "reth/reth/utils/__init__.py")
    alg = _pkg("reth.algorithm")
    R.algorithm = _load("reth.algorithm.algorithm", "reth/reth/algorithm/algorithm.py")
    alg.Algorithm = R.algorithm.Algorithm
    _load("reth.algorithm.util", "reth/reth/algorithm/util.py")
    _pkg("reth.algorithm.dqn")
    R.dqn_model = _load("reth.algorithm.dqn.dqn_model", "reth/reth/algorithm/dqn/dqn_model.py")
    R.dqn_solver = _load("reth.algorithm.dqn.dqn_solver", "reth/reth/algorithm/dqn/dqn_solver.py")
    R.gym = sys.modules["gym"]
    return R


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# ----------------------------------------------------------------------------- sum-tree
def tree_state(t):
    return t._sum.copy(), t._min.copy(), t._val.copy()


def gen_sumtree_small(R):
    out = {}
    rng = np.random.default_rng(1)
    NumbaSumTree = R.sumtree.NumbaSumTree
    find = R.sumtree._numba_find_index

    def record(tag, t, updates, targets, sample_b=None, seed=0):
        s, m, v = tree_state(t)
        out[f"{tag}/capacity"] = np.int64(t.capacity)
        out[f"{tag}/sum"], out[f"{tag}/min"], out[f"{tag}/val"] = s, m, v
        out[f"{tag}/tree_min"] = np.float64(t.min())
        out[f"{tag}/targets"] = np.asarray(targets, np.float64)
        out[f"{tag}/find"] = np.array([find(t._tree, w) for w in targets], np.int64)
        for k, (idx, w) in enumerate(updates):
            out[f"{tag}/upd{k}_idx"] = np.asarray(idx, np.int64)
            out[f"{tag}/upd{k}_w"] = np.asarray(w, np.float64)
        out[f"{tag}/n_upd"] = np.int64(len(updates))
        if sample_b:
            np.random.seed(seed)
            u = np.random.random_sample(sample_b)
            np.random.seed(seed)
            idx, vals = t.sample(sample_b)
            out[f"{tag}/sample_u"], out[f"{tag}/sample_idx"], out[f"{tag}/sample_val"] = u, idx, vals

    def run(cap, updates):
        t = NumbaSumTree(cap)
        for idx, w in updates:
            t.update(np.asarray(idx), np.asarray(w))
        return t

    # A: C=10, all ones -> in-order mass mapping [7,3,8,1,9,4,0,5,2,6]
    ups = [(np.arange(10), np.ones(10))]
    t = run(10, ups)
    tg = [k + 0.5 for k in range(10)] + [10.0, 10.5, 100.0, 0.0, 9.999995, 2.99999]
    record("c10", t, ups, tg, sample_b=10, seed=3)
    # B: C=5, targets at/after the total (return last in-order node)
    ups = [(np.arange(5), np.array([0.5, 1.5, 0.25, 2.0, 1.0]))]
    t = run(5, ups)
    record("c5", t, ups, [0.0, 0.49, 0.5, 5.25, 5.2499999, 6.0, 1e9], sample_b=5, seed=4)
    # C: C=1, degenerate
    ups = [(np.array([0]), np.array([0.7]))]
    t = run(1, ups)
    record("c1", t, ups, [0.0, 0.69, 0.7, 5.0], sample_b=3, seed=5)
    # D: C=1000, partial fill with exact zeros, then duplicate-heavy updates touching
    #    never-filled slots (exercises the min() seed quirk, sumtree.py:11-19)
    w0 = rng.random(600)
    w0[::37] = 0.0
    up1 = (np.arange(600), w0)
    idx2 = rng.integers(0, 1000, 300)
    idx2[:20] = idx2[20:40]  # forced duplicates (last writer wins)
    w2 = rng.random(300)
    w2[::11] = 0.0
    ups = [up1, (idx2, w2)]
    t = run(1000, ups)
    tot = t.sum()
    tg = list(rng.random(50) * tot) + [tot, tot * (1 - 1e-12), tot + 1.0, 0.0]
    record("c1000", t, ups, tg, sample_b=64, seed=6)
    # E: C=3000, 1200 filled in FIFO chunks of 64 (append path), then 512 updates with
    #    duplicates (learner path) -- SURVEY App. A.2 probe shape
    ups = []
    for s in range(0, 1200, 64):
        n = min(64, 1200 - s)
        ups.append((np.arange(s, s + n), (rng.random(n).astype(np.float32) + np.float32(1e-6)) ** 0.5))
    idx = rng.integers(0, 1200, 512)
    ups.append((idx, rng.random(512)))
    t = run(3000, ups)
    tg = list(rng.random(100) * t.sum())
    record("c3000", t, ups, tg, sample_b=512, seed=7)
    # F: C=4097 (ragged last level), full random then a sparse re-update incl. zeros
    ups = [(np.arange(4097), rng.random(4097)), (rng.integers(0, 4097, 1000), np.where(rng.random(1000) < 0.1, 0.0, rng.random(1000)))]
    t = run(4097, ups)
    record("c4097", t, ups, list(rng.random(200) * t.sum()), sample_b=128, seed=8)
    np.savez_compressed(os.path.join(OUT, "sumtree_small.npz"), **out)


def gen_sumtree_large(R):
    """Pong-depth tree (C=2^20, 21 levels): FIFO fill in 256-row appends + 40 learner
    updates of 512 indices.  Inputs are regenerated from the seed by the test
    (np.random.default_rng is stable); outputs stored as hashes + one sampled batch."""
    seed, cap, chunk, n_learn, B = 20, 1 << 20, 256, 40, 512
    rng = np.random.default_rng(seed)
    t = R.sumtree.NumbaSumTree(cap)
    per_norm = lambda w: (w + np.float32(1e-6)) ** np.float32(0.5)
    for s in range(0, cap, chunk):
        td = rng.random(chunk, dtype=np.float32)
        t.update(np.arange(s, s + chunk, dtype=np.int64), per_norm(td))
    for _ in range(n_learn):
        idx = rng.integers(0, cap, B)
        td = rng.random(B, dtype=np.float32) * np.float32(3.0)
        t.update(idx, per_norm(td))
    np.random.seed(seed)
    u = np.random.random_sample(B)
    np.random.seed(seed)
    sidx, sval = t.sample(B)
    out = dict(seed=np.int64(seed), capacity=np.int64(cap), chunk=np.int64(chunk),
               n_learn=np.int64(n_learn), batch=np.int64(B), sample_u=u,
               sample_idx=sidx, sample_val=sval, total=np.float64(t.sum()),
               tree_min=np.float64(t.min()))
    out["sha_sum"], out["sha_min"], out["sha_val"] = sha(t._sum), sha(t._min), sha(t._val)
    np.savez_compressed(os.path.join(OUT, "sumtree_large.npz"), **out)


# ----------------------------------------------------------------------------- PER
def gen_per(R):
    out = {}
    rng = np.random.default_rng(2)
    for alpha, tag in ((0.5, "a05"), (0.6, "a06")):
        s = R.per.PERSampler(2000, alpha=alpha, beta="0.4,1,2000000")
        w = rng.random(4000, dtype=np.float32) * np.float32(4.0)
        w[:5] = [0.0, 1e-7, 1.0, 3.5, 1e-30]
        norm = s._normalize_weights(w)
        out[f"{tag}/w"], out[f"{tag}/norm"] = w, norm
        # append 1500 rows in 64-row messages, then 8 learner steps (on_step + update)
        for st in range(0, 1500, 64):
            n = min(64, 1500 - st)
            s.update(np.arange(st, st + n, dtype=np.int32), w[st:st + n])
        betas, samples = [], []
        for k in range(8):
            np.random.seed(100 + k)
            u = np.random.random_sample(64)
            np.random.seed(100 + k)
            idx, isw = s.sample(64)
            out[f"{tag}/s{k}_u"], out[f"{tag}/s{k}_idx"], out[f"{tag}/s{k}_isw"] = u, idx, isw
            betas.append(s.beta.value())
            s.on_step()
            s.update(idx, w[1500 + 64 * k: 1564 + 64 * k])
        out[f"{tag}/betas"] = np.array(betas)
        out[f"{tag}/alpha_f32"] = np.float32(alpha)
        out[f"{tag}/final_sha_sum"] = sha(s.sumtree._sum)
        out[f"{tag}/final_sha_val"] = sha(s.sumtree._val)
        out[f"{tag}/final_sum"] = np.float64(s.sumtree.sum())
        out[f"{tag}/final_min"] = np.float64(s.sumtree.min())
    np.savez_compressed(os.path.join(OUT, "per.npz"), **out)


# ----------------------------------------------------------------------------- schedule / FIFO
def gen_schedule_fifo(R):
    S = R.schedule.Schedule
    steps = [0, 1, 2, 3, 10, 999, 1000, 1001, 123457, 1999999, 2000000, 2000001, 5000000]
    res = {"steps": steps, "cases": []}
    for spec in ["0.4,1,2000000", "linear,0.4,1,2000000", "exp,1,0.01,1000", "1,0.01,100000", 0.5, 3]:
        sch = S.from_str(spec)
        vals = [sch.value(k) for k in steps]
        seq = [sch.step() for _ in range(5)]
        res["cases"].append({"spec": spec, "value": [float(x).hex() for x in vals],
                             "step_seq": [float(x).hex() for x in seq]})
    bad = []
    for spec in ["0.5", "a,b", "cubic,0,1,10"]:
        try:
            S.from_str(spec)
            bad.append({"spec": spec, "raises": False})
        except Exception:
            bad.append({"spec": spec, "raises": True})
    res["invalid"] = bad
    fifo = R.fifo.FIFOPolicy(10)
    res["fifo_capacity"] = 10
    res["fifo_requests"] = [3, 4, 7, 10, 1]
    res["fifo_indices"] = [fifo.get_indices(n).tolist() for n in res["fifo_requests"]]
    with open(os.path.join(OUT, "schedule_fifo.json"), "w") as f:
        json.dump(res, f, indent=1)


# ----------------------------------------------------------------------------- n-step
def gen_nstep(R):
    """Streams through the reference NStepAdder (numpy-2 / NEP 50 scalar semantics in this
    container: the f32 product t_gamma*r stays f32)."""
    out = {"numpy_version": np.array(np.__version__)}
    rng = np.random.default_rng(3)
    streams = {
        "nodone": np.zeros(12),
        "done_t2": np.array([0, 0, 1, 0, 0, 0, 0, 0]),
        "done_each3": np.array([0, 0, 1] * 5),
        "done_adjacent": np.array([0, 1, 1, 0, 1, 0, 0, 1, 0, 0]),
        "random": (rng.random(300) < 0.08).astype(np.float64),
    }
    for n_step in (1, 3, 5):
        for name, dones in streams.items():
            tag = f"n{n_step}/{name}"
            T = len(dones)
            rewards = np.where(rng.random(T) < 0.5, rng.choice([-1.0, 1.0], T), rng.random(T) * 2 - 1).astype(np.float32)
            if name == "done_t2":
                rewards[:] = 1.0
            actions = rng.integers(0, 6, T)
            adder = R.rutils.NStepAdder(0.99, n_step)
            rows = []
            for t in range(T):
                row = adder.push(np.asarray(t, "f4"), np.asarray(actions[t], "i8"), np.asarray(rewards[t], "f4"),
                                 np.asarray(t + 1000, "f4"), np.asarray(dones[t], "f4"))
                if row is not None:
                    rows.append((t, float(row[0]), int(row[1]), np.float32(row[2]), float(row[3]), float(row[4])))
            out[f"{tag}/rewards"], out[f"{tag}/actions"], out[f"{tag}/dones"] = rewards, actions.astype(np.int64), dones.astype(np.float32)
            arr = np.array([(r[0], r[1], r[2], r[4], r[5]) for r in rows], dtype=np.float64).reshape(-1, 5)
            out[f"{tag}/emit_t"] = arr[:, 0].astype(np.int64)
            out[f"{tag}/emit_s0"] = arr[:, 1].astype(np.int64)
            out[f"{tag}/emit_a"] = arr[:, 2].astype(np.int64)
            out[f"{tag}/emit_r"] = np.array([r[3] for r in rows], np.float32)
            out[f"{tag}/emit_s1"] = (arr[:, 3] - 1000).astype(np.int64)
            out[f"{tag}/emit_done"] = arr[:, 4].astype(np.float32)
    np.savez_compressed(os.path.join(OUT, "nstep.npz"), **out)


# ----------------------------------------------------------------------------- DQN
def _param_stats(net):
    names, s1, s2, head = [], [], [], []
    for k, v in net.state_dict().items():
        v = v.detach().double().flatten()
        names.append(k)
        s1.append(float(v.sum()))
        s2.append(float((v * v).sum()))
        h = np.full(16, np.nan, np.float32)
        x = v[:16].float().numpy()
        h[: len(x)] = x
        head.append(h)
    return names, np.array(s1), np.array(s2), head


def gen_dqn(R):
    import torch
    torch.set_num_threads(4)
    gym = R.gym
    DQNSolver = R.dqn_solver.DQNSolver

    # --- Pong-shaped conv net, A=6, B=8 (apex-dqn config.yaml hyper-parameters)
    for B, tag in ((8, "pong_b8"), (32, "pong_b32")):
        seed = 1234 + B
        torch.manual_seed(seed)
        solver = DQNSolver(gym.spaces.Box(0, 255, (4, 84, 84)), gym.spaces.Discrete(6), gamma=0.99,
                           clip_value=40, double_q=True, dueling=True, learning_rate=1e-4,
                           adam_epsilon=1.5e-4, update_target_interval=100, device="cpu", n_step=3)
        rng = np.random.default_rng(seed)
        s0 = rng.integers(0, 256, (B, 4, 84, 84), dtype=np.uint8)
        s1 = rng.integers(0, 256, (B, 4, 84, 84), dtype=np.uint8)
        a = rng.integers(0, 6, B).astype(np.int64)
        r = rng.choice(np.array([-1.0, 0.0, 1.0], np.float32), B).astype(np.float32)
        done = (rng.random(B) < 0.25).astype(np.float32)
        isw = rng.random(B) + 0.2  # f64, as the sampler produces
        batch = [s0.astype("f4"), a, r, s1.astype("f4"), done]
        out = dict(seed=np.int64(seed), s0=s0, s1=s1, a=a, r=r, done=done, isw=isw)
        names, p1, p2, head = _param_stats(solver.q_network)
        out["init_sum"], out["init_sq"] = p1, p2
        with torch.no_grad():
            tq = lambda x: torch.as_tensor(x)
            out["q_s0"] = solver.q_network(tq(batch[0])).numpy()
            out["q_s1_online"] = solver.q_network(tq(batch[3])).numpy()
            out["q_s1_target"] = solver.target_q_network(tq(batch[3])).numpy()
            out["td"] = solver._calc_td_error(batch).numpy()
        out["calc_loss"] = solver.calc_loss(batch).numpy()
        out["act0"] = np.int64(solver.act(batch[0][0]))
        # two updates (second one exercises Adam state); record returned |td| and params
        for k in range(2):
            out[f"upd{k}_abs_td"] = solver.update(batch, weights=isw).numpy()
            names, p1, p2, head = _param_stats(solver.q_network)
            out[f"upd{k}_sum"], out[f"upd{k}_sq"] = p1, p2
            out[f"upd{k}_head"] = np.stack(head)
        out["param_names"] = np.array(names)
        np.savez_compressed(os.path.join(OUT, f"dqn_{tag}.npz"), **out)

    # --- CartPole MLP, A=2, B=64: full post-update state_dict
    seed = 77
    torch.manual_seed(seed)
    solver = DQNSolver(gym.spaces.Box(-1, 1, (4,)), gym.spaces.Discrete(2), gamma=0.99, clip_value=40,
                       double_q=True, dueling=True, learning_rate=1e-4, update_target_interval=200,
                       device="cpu")
    rng = np.random.default_rng(seed)
    B = 64
    s0 = rng.standard_normal((B, 4)).astype(np.float32)
    s1 = rng.standard_normal((B, 4)).astype(np.float32)
    a = rng.integers(0, 2, B).astype(np.int64)
    r = np.ones(B, np.float32)
    done = (rng.random(B) < 0.1).astype(np.float32)
    out = dict(seed=np.int64(seed), s0=s0, s1=s1, a=a, r=r, done=done)
    for k, v in solver.q_network.state_dict().items():
        out[f"init/{k}"] = v.numpy().copy()
    batch = [s0, a, r, s1, done]
    out["td"] = solver._calc_td_error(batch).detach().numpy()
    for k in range(3):  # no IS weights (uniform replay, examples/dqn/run.py:29)
        out[f"upd{k}_abs_td"] = solver.update(batch).numpy()
    for k, v in solver.q_network.state_dict().items():
        out[f"final/{k}"] = v.numpy().copy()
    np.savez_compressed(os.path.join(OUT, "dqn_cartpole_b64.npz"), **out)


def gen_dqn_full(R):
    """the apex learner's own batch sizes: B = 512, A = 6 (Pong, test/apex-dqn/config.yaml:2)
    and B = 64, A = 9 (the reference config's BeamRider, config.yaml:8).  Two reference
    updates (dqn_solver.py:104-124) on one batch; the FULL state_dict after each, stored as
    float16 deltas from the seeded initial weights (|delta| <= ~3e-4 after two Adam steps of
    lr 1e-4, so the float16 rounding is <= 1.5e-7), plus every |td| returned.

    The same reference code is also run in float64 (networks, Adam and the batch in double:
    ensure_tensor's torch.float cast redirected to float64) -- the exact update the fp32 runs
    approximate.  Its deltas (float16) and the reference fp32 run's own per-tensor max error
    against it are stored: the reference's fp32 CPU update is itself up to ~1.6e-5 from the
    exact one on conv1's weight after two updates (Adam's eps = 1.5e-4 amplifies the fp32
    gradient rounding of near-zero gradients), so a parity test needs that yardstick.
    The frames come from tests/golden/dqn_batch.py (seed -> SHA-256 here)."""
    import torch

    sys.path.insert(0, OUT)
    from dqn_batch import apex_batch, frames_sha

    torch.set_num_threads(8)
    gym = R.gym

    def run(seed, B, A, f64):
        torch.manual_seed(seed)
        solver = R.dqn_solver.DQNSolver(gym.spaces.Box(0, 255, (4, 84, 84)), gym.spaces.Discrete(A), gamma=0.99,
                                        clip_value=40, double_q=True, dueling=True, learning_rate=1e-4,
                                        adam_epsilon=1.5e-4, update_target_interval=100, device="cpu", n_step=3)
        # the first update's gradient as the reference's update hands it to clip_grad_norm_
        # (dqn_solver.py:117-119): recorded by a pass-through wrapper, with the norm it returns
        names = {id(p): n for n, p in solver.q_network.named_parameters()}
        grads = {}
        clip_orig = torch.nn.utils.clip_grad_norm_

        def clip_rec(params, max_norm, *a, **k):
            params = list(params)
            if not grads:
                grads.update({names[id(p)]: p.grad.detach().double().clone().numpy() for p in params})
            norm = clip_orig(params, max_norm, *a, **k)
            grads.setdefault("__norm__", float(norm))
            return norm

        torch.nn.utils.clip_grad_norm_ = clip_rec
        orig = R.dqn_solver.ensure_tensor
        if f64:
            solver.q_network.double()
            solver.target_q_network.double()
            solver.optimizer = torch.optim.Adam(solver.q_network.parameters(), lr=1e-4, eps=1.5e-4)
            R.dqn_solver.ensure_tensor = lambda arr, dtype, device, non_blocking=True: orig(
                arr, torch.float64 if dtype == torch.float else dtype, device)
        try:
            s0, s1, a, r, done, isw = apex_batch(seed, B, A)
            batch = [s0.astype("f4"), a, r, s1.astype("f4"), done]
            init = {k: v.detach().clone() for k, v in solver.q_network.state_dict().items()}
            res = []
            for _ in range(2):
                tgt = None
                if f64:  # the TD target r + gamma^n Q_target(s1, argmax_a Q(s1, a)) (1 - done) of this
                    # update (dqn_solver.py:84-96), in float64: the scale the north-star 1e-5 applies to
                    with torch.no_grad():
                        x1 = torch.as_tensor(s1).double()
                        best = solver.q_network(x1).argmax(1, keepdim=True)
                        nxt = solver.target_q_network(x1).gather(1, best).view(-1)
                        tgt = (torch.as_tensor(r).double() + 0.99 ** 3 * nxt *
                               (1 - torch.as_tensor(done).double())).numpy()
                td = solver.update(batch, weights=isw)
                res.append((td.double().numpy(), {n: (v.detach().double() - init[n].double()).numpy()
                                                  for n, v in solver.q_network.state_dict().items()}, tgt))
        finally:
            R.dqn_solver.ensure_tensor = orig
            torch.nn.utils.clip_grad_norm_ = clip_orig
        return init, res, (s0, s1, a, r, done, isw), grads

    def margins(seed, B, A):
        """float64 decision margins of the first update's forward, relative to sum |x| |w|: the
        FC1 ReLUs of the s0 rows (a flipped unit there moves a whole row of FC1's gradient:
        one flip at a relative margin of 1.3e-8 -- below fp32 rounding -- put 2e-3 into
        fc_adv.0.weight's gradient on seed 4760) and the double-Q argmax of the online heads
        on s1 (top-2 gap relative to the heads' magnitude)"""
        torch.manual_seed(seed)
        solver = R.dqn_solver.DQNSolver(gym.spaces.Box(0, 255, (4, 84, 84)), gym.spaces.Discrete(A), gamma=0.99,
                                        clip_value=40, double_q=True, dueling=True, learning_rate=1e-4,
                                        adam_epsilon=1.5e-4, update_target_interval=100, device="cpu", n_step=3)
        net = solver.q_network.double()
        s0, s1, *_ = apex_batch(seed, B, A)
        with torch.no_grad():
            f = net.features(torch.as_tensor(np.concatenate([s0, s1])).double()).reshape(2 * B, -1)
            relu = np.inf
            for fc in (net.fc_adv[0], net.fc_value[0]):
                pre = f[:B] @ fc.weight.t() + fc.bias
                scale = f[:B].abs() @ fc.weight.abs().t() + fc.bias.abs()
                relu = min(relu, float((pre.abs() / scale).min()))
            q1 = net(torch.as_tensor(s1).double())
            top = torch.topk(q1, 2, dim=1).values
            gap = float(((top[:, 0] - top[:, 1]) / q1.abs().max(1).values.clamp_min(1e-30)).min())
        return relu, gap

    for B, A, tag in ((512, 6, "pong_b512"), (64, 9, "beamrider_b64")):
        # the batch + seeded init is screened: of 40 candidate seeds the one whose closest FC1
        # ReLU / double-Q argmax decision of the exact update lies farthest from its threshold
        # (~1e-6 relative at B = 512, where a 512 x 1024 FC1 has a few pre-activations per 1e-6
        # of relative margin): decisions closer than fp32 rounding are coin flips that any two
        # fp32 summation orders -- the reference's own CPU run included -- may take differently
        cands = []
        for k in range(40):
            sd = 4242 + B + A + 1000 * k
            cands.append((min(margins(sd, B, A)), sd))
            print(f"  dqn_{tag}: seed {sd} min margin {cands[-1][0]:.2e}", flush=True)
        seed = max(cands)[1]
        relu_m, gap_m = margins(seed, B, A)
        init, r32, (s0, s1, a, r, done, isw), g32 = run(seed, B, A, False)
        _, r64, _, g64 = run(seed, B, A, True)
        out = dict(seed=np.int64(seed), B=np.int64(B), A=np.int64(A), frames_sha=np.array(frames_sha(s0, s1)),
                   a=a, r=r, done=done, isw=isw, param_names=np.array(list(init)))
        out["init_sum"] = np.array([float(v.double().sum()) for v in init.values()])
        out["margin_fc1_relu"], out["margin_argmax"] = np.float64(relu_m), np.float64(gap_m)
        for k in range(2):
            out[f"upd{k}_abs_td"] = r32[k][0].astype(np.float32)
            out[f"upd{k}_abs_td64"] = r64[k][0]
            out[f"upd{k}_target64"] = r64[k][2]
            rel = np.abs(r32[k][0] - r64[k][0]) / np.maximum(1.0, np.abs(r64[k][2]))
            print(f"  dqn_{tag} update {k}: reference fp32 |td| error / max(1, |target|) <= {rel.max():.2e}")
            errs = []
            for name in init:
                d32, d64 = r32[k][1][name], r64[k][1][name]
                assert np.abs(d32).max() < 6e-4 and np.abs(d64).max() < 6e-4, name
                out[f"upd{k}_64/{name}"] = d64.astype(np.float16)  # the exact update; the fp32 run
                errs.append(np.abs(d32 - d64).max())               # is kept as its distance only
            out[f"upd{k}_ref32_err"] = np.array(errs)  # per tensor: max |reference fp32 - exact|
        # the first update's gradient (before clipping) of the exact run, float32: every element of
        # every tensor but FC1's two weights, of which every GRAD_ROW_STRIDE-th row (a row of FC1's
        # weight gradient is one hidden unit's: sum_b gh1[b, i] feat[b, :]); the fp32 run's distance
        # per tensor over the same elements; both runs' total norms (clip_grad_norm_'s return)
        gerr, gmax = [], []
        for name in init:
            sel = (slice(None, None, GRAD_ROW_STRIDE),) if name.endswith(".0.weight") and name.startswith("fc_") \
                else (Ellipsis,)
            e64, e32 = g64[name][sel], g32[name][sel]
            out[f"grad0_64/{name}"] = e64.astype(np.float32)
            gerr.append(np.abs(e32 - e64).max())
            gmax.append(np.abs(e64).max())
        out["grad0_ref32_err"], out["grad0_absmax"] = np.array(gerr), np.array(gmax)
        out["grad0_row_stride"] = np.int64(GRAD_ROW_STRIDE)
        out["grad0_norm64"], out["grad0_norm32"] = np.float64(g64["__norm__"]), np.float64(g32["__norm__"])
        print(f"  dqn_{tag} grad norm {g64['__norm__']:.6e} (fp32 run {g32['__norm__']:.6e}); fp32 grad error / "
              f"max|g| per tensor: " + " ".join(f"{e / max(m, 1e-30):.1e}" for e, m in zip(gerr, gmax)))
        np.savez_compressed(os.path.join(OUT, f"dqn_{tag}.npz"), **out)


GRAD_ROW_STRIDE = 8


# ----------------------------------------------------------------------------- samplers / buffers
def _load_buffers(R):
    """reth.buffer (NumpyBuffer, PrioritizedBuffer with its own NumbaSumTree) and the
    Uniform / FIFO samplers; readerwriterlock is absent -> a no-op lock shim"""
    import contextlib

    rw = types.ModuleType("readerwriterlock")

    class _Lock:
        def gen_wlock(self):
            return contextlib.nullcontext()

        def gen_rlock(self):
            return contextlib.nullcontext()

    rw.rwlock = types.SimpleNamespace(RWLockWrite=_Lock)
    sys.modules["readerwriterlock"] = rw
    sys.modules["readerwriterlock.rwlock"] = rw.rwlock
    _pkg("reth.buffer")
    R.buf = _load("reth.buffer.buffer", "reth/reth/buffer/buffer.py")
    R.bsum = _load("reth.buffer.sumtree", "reth/reth/buffer/sumtree.py")
    R.pbuf = _load("reth.buffer.prioritized_buffer", "reth/reth/buffer/prioritized_buffer.py")
    R.uni = _load("rb.sampler.uniform_sampler", "reth_buffer/reth_buffer/sampler/uniform_sampler.py")
    R.fifos = _load("rb.sampler.fifo_sampler", "reth_buffer/reth_buffer/sampler/fifo_sampler.py")


def gen_buffers(R):
    _load_buffers(R)
    out = {}
    rng = np.random.default_rng(77)
    # FIFOSampler (capacity 50): appends (FIFO-policy slots) and explicit updates, samples
    cap = 50
    fs, pol = R.fifos.FIFOSampler(cap), R.fifo.FIFOPolicy(cap)
    ops = [("a", 30), ("s", 10), ("u", 40), ("s", 25), ("a", 45), ("s", 45), ("u", 7), ("s", 3)]
    for k, (op, n) in enumerate(ops):
        if op == "s":
            out[f"fifo{k}_ready"] = np.array(fs.ready_sample(n))
            i, w = fs.sample(n)
            out[f"fifo{k}_idx"], out[f"fifo{k}_w"] = np.asarray(i, np.int64), np.asarray(w, np.float64)
        else:
            idx = pol.get_indices(n) if op == "a" else rng.integers(0, cap, n)
            w = rng.random(n).astype(np.float32)
            out[f"fifo{k}_in_idx"], out[f"fifo{k}_in_w"] = np.asarray(idx, np.int64), w
            fs.update(idx, w)
    out["fifo_ops"] = np.array([f"{op}{n}" for op, n in ops])
    # UniformSampler (capacity 64): the list fills to exactly capacity, then ignores updates;
    # sample positions recorded by replaying numpy's global stream
    cap = 64
    us, pol = R.uni.UniformSampler(cap), R.fifo.FIFOPolicy(cap)
    np.random.seed(5)
    ops = [("a", 20), ("u", 30), ("s", 16), ("a", 14), ("s", 32), ("a", 10), ("u", 5), ("s", 40)]
    for k, (op, n) in enumerate(ops):
        if op == "s":
            st = np.random.get_state()
            pos = np.random.choice(us.tail, n)
            np.random.set_state(st)
            i, w = us.sample(n)
            out[f"uni{k}_pos"], out[f"uni{k}_tail"] = pos.astype(np.int64), np.array(us.tail)
            out[f"uni{k}_idx"], out[f"uni{k}_w"] = np.asarray(i, np.int64), np.asarray(w)
        else:
            idx = pol.get_indices(n) if op == "a" else rng.integers(0, cap, n)
            out[f"uni{k}_in_idx"] = np.asarray(idx, np.int64)
            us.update(idx, np.ones(n, np.float32))
    out["uni_ops"] = np.array([f"{op}{n}" for op, n in ops])
    # NumpyBuffer (capacity 10, circular) + DynamicSizeBuffer growth
    nb = R.buf.NumpyBuffer(10)
    rows = lambda n: [rng.standard_normal((n, 4)), rng.integers(0, 6, n), rng.random(n) < 0.3]
    k = 0
    for kind, n in [("one", 1), ("one", 1), ("one", 1), ("batch", 5), ("batch", 6), ("one", 1), ("batch", 10)]:
        r = rows(n)
        for c, col in enumerate(r):
            out[f"nb{k}_in{c}"] = col
        if kind == "one":
            ret = np.array([nb.append([col[0] for col in r])])
        else:
            ret = np.asarray(nb.append_batch(r))
        out[f"nb{k}_ret"], out[f"nb{k}_tail"], out[f"nb{k}_size"] = ret.astype(np.int64), np.array(nb._tail), np.array(nb.size)
        k += 1
    for c, col in enumerate(nb.data):
        out[f"nb_data{c}"] = col
    out["nb_steps"] = np.array(k)
    dyn = R.buf.DynamicSizeBuffer(4)
    caps = []
    for n in (1, 1, 1, 1, 1, 3, 10):
        r = rows(n)
        if n == 1:
            dyn.append([col[0] for col in r])
        else:
            dyn.append_batch(r)
        caps.append((dyn.capacity, dyn.size))
    out["dyn_caps"] = np.array(caps, np.int64)
    # PrioritizedBuffer (reth.buffer): alpha 0.6, beta "0.4,1,1000", capacity 100
    pb = R.pbuf.PrioritizedBuffer(100, alpha=0.6, beta="0.4,1,1000")
    d = lambda n: [rng.standard_normal((n, 3)).astype(np.float32), rng.integers(0, 4, n)]
    # (PrioritizedBuffer.append of one row fails in the reference: the 0-d index/weight
    # arrays it passes to _numba_update have no len(), prioritized_buffer.py:31-35)
    seq = [("batch_w", 60), ("batch", 50), ("sample", 32), ("sample", 32), ("update", 40), ("sample", 32),
           ("batch_w", 20), ("sample", 64)]
    np.random.seed(9)
    for k, (op, arg) in enumerate(seq):
        if op == "batch_w":
            r, w = d(arg), rng.random(arg)
            out[f"pb{k}_d0"], out[f"pb{k}_d1"], out[f"pb{k}_w"] = r[0], r[1], w
            pb.append_batch(r, weights=w)
        elif op == "batch":
            r = d(arg)
            out[f"pb{k}_d0"], out[f"pb{k}_d1"] = r[0], r[1]
            pb.append_batch(r)
        elif op == "one":
            r = d(1)
            out[f"pb{k}_d0"], out[f"pb{k}_d1"] = r[0], r[1]
            out[f"pb{k}_w"] = np.array(np.nan if arg is None else arg)
            pb.append([r[0][0], r[1][0]], arg)
        elif op == "update":
            idx, w = rng.integers(0, 100, arg), rng.random(arg).astype(np.float32)
            out[f"pb{k}_idx"], out[f"pb{k}_w"] = idx, w
            pb.update_priorities(idx, w)
        else:
            st = np.random.get_state()
            u = np.random.random_sample(arg)
            np.random.set_state(st)
            data, idx, w = pb.sample(arg)
            out[f"pb{k}_u"], out[f"pb{k}_idx"], out[f"pb{k}_isw"] = u, np.asarray(idx), np.asarray(w)
            out[f"pb{k}_rows0"] = data[0]
        out[f"pb{k}_sum"] = pb.sumtree._sum.copy()
    out["pb_ops"] = np.array([op for op, _ in seq])
    np.savez_compressed(os.path.join(OUT, "buffers.npz"), **out)


# ----------------------------------------------------------------------------- wire format
def gen_pack(R):
    """reth_buffer/utils/pack.py messages (uncompressed; lz4 and loguru are absent -> stubs),
    with time.time() pinned so the bytes are reproducible"""
    lz4 = types.ModuleType("lz4")
    lz4.frame = types.ModuleType("lz4.frame")
    sys.modules["lz4"], sys.modules["lz4.frame"] = lz4, lz4.frame
    loguru = types.ModuleType("loguru")
    loguru.logger = types.SimpleNamespace(info=lambda *a, **k: None, warning=lambda *a, **k: None)
    sys.modules["loguru"] = loguru
    pack = _load("rb.utils.pack", "reth_buffer/reth_buffer/utils/pack.py")
    pack.time = types.SimpleNamespace(time=lambda: 1234.5)
    rng = np.random.default_rng(11)
    out = {}
    # a Client.append message as test/apex-dqn/worker.py sends it (float32 frames)
    n = 6
    s0 = rng.integers(0, 256, (n, 4, 10, 12)).astype("f4")
    s1 = rng.integers(0, 256, (n, 4, 10, 12)).astype("f4")
    a = rng.integers(0, 6, n).astype("i8")
    r = rng.choice(np.array([-1, 0, 1], "f4"), n)
    done = (rng.random(n) < 0.3).astype("f4")
    w = rng.random(n).astype("f4")
    rows = [pack.serialize([c[i, ...] for c in (s0, a, r, s1, done)]) for i in range(n)]  # client.py:27-33
    msg = pack.serialize([rows, w])
    out.update(app_s0=s0, app_s1=s1, app_a=a, app_r=r, app_done=done, app_w=w,
               app_msg=np.frombuffer(bytes(msg), np.uint8))
    # a generic nested object (dict / list / bytes / scalars / Fortran array / 0-d array)
    obj = {"x": [np.arange(10, dtype="i4"), b"raw-bytes", 3, "s", 2.5],
           "f": np.asfortranarray(rng.standard_normal((3, 4))), "z": np.array(7.0, "f8"), "e": [[], {}]}
    out["obj_msg"] = np.frombuffer(bytes(pack.serialize(obj)), np.uint8)
    out["obj_x0"], out["obj_f"] = obj["x"][0], obj["f"]
    # update_priorities message
    out["upd_msg"] = np.frombuffer(bytes(pack.serialize([np.arange(5), w[:5], True])), np.uint8)
    np.savez_compressed(os.path.join(OUT, "pack.npz"), **out)


def main():
    R = load_reference()
    which = sys.argv[1:] or ["sumtree_small", "sumtree_large", "per", "schedule_fifo", "nstep", "dqn", "buffers", "pack"]
    for w in which:
        print("generating", w, flush=True)
        globals()[f"gen_{w}"](R)
    print("done")


if __name__ == "__main__":
    main()
