"""Ape-X DQN Pong benchmark: env-steps/s + learner updates/s on N MI355X (one process each).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    (N > 1 under: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)

Workload (BASELINE.json configs[1]): per GPU 256 vectorised actors on a
synthetic Pong-shaped env (uint8 4x84x84 frame stacks, A = 6; ALE is not on the box), a 1 M
transition prioritized replay shard in HBM pre-filled to capacity, B = 512, n = 3,
gamma = 0.99, alpha = 0.5, beta 0.4 -> 1 over 2 M, Adam lr 1e-4 eps 1.5e-4, clip 40, target
every 100 updates, weights published every 10 (test/apex-dqn/config.yaml).  One step = 256
env steps (act, env, n-step, priorities, insert) + one learner update (sample, gather, TD,
backward, Adam, priority write-back), all fp32 / fp64 as in the reference.  N > 1 is weak
scaling: every GPU runs the same per-GPU workload and the learner gradients are averaged
with one RCCL all-reduce per update.

The JSON line carries
  roofline:        the dominant kernel of the step: whichever of conv2 / conv3 forward has the
                   most kernel time per iteration (conv_iteration_alone: its learner, target
                   and actor launches timed alone), measured in the learner's [s0; s1] pass
                   live over the timed region with HIP events on the learner stream (the
                   learner graph is cut once, around the conv2 + conv3 launches); achieved =
                   algorithmic FLOPs per launch / mean launch duration, against the fp32 MFMA
                   peak (dtype f32); an exact-split bf16 kernel (k_conv_x9) also reports the
                   bf16 MFMA FLOPs it issues against the bf16 peak (mfma_issue)
  roofline_conv2 / roofline_conv3: both conv kernels, timed the same way
  roofline_gather: the replay gather (k_copy_rows), HBM-bound, timed live the same way
  roofline_conv1:  conv1 on uint8 stacks (k_conv1_u8_bf16x3) alone, against the bf16 MFMA peak
                   of the instruction it issues (three exact-split bf16 products per fp32 one)
  cpu_baseline:    the same step on the host cores (oracle restatement of the replay/tree/
                   n-step path + torch-CPU Q-network), bounded sample, rank 0 at N = 1.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

STACK = 4 * 84 * 84
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3  # fp32-input MFMA (= the fp32 vector peak)
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA
# BASELINE.json configs[1] / configs[3] (the metric's workload at N = 1 / N > 1), the weak
# replication of configs[1], and configs[2] (a scale case, not the bench line)
WORKLOADS = {
    # configs[1] at N = 1; configs[3] at N > 1: the reference's apex-dqn deployment sharded over
    # the node (test/apex-dqn/trainer.py:52-61: K replay shards of C // K; worker.py:83-99: the
    # actors split over the nodes): 256 / N actors and 1 M / N rows per GPU, one data-parallel
    # learner replica per GPU (RCCL gradient all-reduce), B = 512 per GPU (--faithful: a global
    # 512).  Each learner update is paired with 256 env steps of its shard (actor_steps_per_update
    # = N), the replay ratio configs[1] runs at, so per-GPU work per step is fixed: weak scaling.
    "pong": dict(name="PongNoFrameskip-v4 Ape-X DQN (BASELINE configs[1])",
                 name_node="Pong Ape-X sharded over {n} GPUs (BASELINE configs[3]: 256 actors and 1 M replay rows "
                           "split over the node, data-parallel learner with an RCCL gradient all-reduce)",
                 actors=256, capacity=1_000_000, actions=6, shard=True),
    # configs[1] replicated on every GPU (256 actors and 1 M rows per GPU)
    "pong-weak": dict(name="PongNoFrameskip-v4 Ape-X DQN, BASELINE configs[1] replicated per GPU (256 actors and "
                           "1 M replay rows on every GPU, data-parallel learner)",
                      actors=256, capacity=1_000_000, actions=6, shard=False),
    "breakout": dict(name="BreakoutNoFrameskip-v4 Ape-X (BASELINE configs[2]; replay storage: see "
                          "config.replay_storage -- full uint8 rows, or --frame-store)", actors=2048,
                     capacity=4_000_000, actions=4, shard=False),
}
WORKLOADS["pong-node"] = WORKLOADS["pong"]


def gather_bytes_per_row(frames_u8=False, frame_ids=False):
    """algorithmic bytes of one sampled apex row in rth_replay_gather: read s0/s1 uint8
    stacks + a(8) r(4) done(4); write s0/s1 as float32 channels-last stacks, or -- with the
    HIP conv torso, which reads uint8 stacks itself -- as the uint8 stacks; a r done; 5
    index reads.  frame_ids (frames in place): s0/s1 are the rows' 2 x 4 int32 frame ids,
    read and written as they are"""
    if frame_ids:
        return 2 * (2 * 16 + 8 + 4 + 4) + 5 * 8
    read = 2 * STACK + 8 + 4 + 4
    write = 2 * STACK * (1 if frames_u8 else 4) + 8 + 4 + 4
    return read + write + 5 * 8


def replay_storage(ax):
    """the replay shard's HBM footprint: full uint8 rows, or the frame store + frame-id rows"""
    rep = ax.replay
    rows = sum(c.row_elems * c.dtype.itemsize if not getattr(c, "frames", False) else c.shape[0] * 4
               for c in rep.columns) * rep.capacity
    if rep.frames is None:
        return {"kind": "full rows (uint8 stacks)", "rows_gb": round(rows / 1e9, 2)}
    fb = rep.frames.numel()
    return {"kind": "frame store (each frame once; rows hold frame ids)", "bound": ax.cfg.frame_store_bound,
            "rows_gb": round(rows / 1e9, 3),
            "frames": int(rep.frames.shape[0]), "frame_store_gb": round(fb / 1e9, 2),
            "total_gb": round((rows + fb) / 1e9, 2),
            "full_rows_would_be_gb": round(rep.capacity * (2 * STACK + 16) / 1e9, 2)}


def qnet_flops_per_sample(A=6):
    """multiply-adds x2 of the Nature-DQN dueling net at 84x84"""
    macs = 32 * 20 * 20 * 4 * 8 * 8 + 64 * 9 * 9 * 32 * 4 * 4 + 64 * 7 * 7 * 64 * 3 * 3 + 3136 * 256 * 2 + 256 * (A + 1)
    return 2 * macs


def conv1_roofline(ax, slot_cols, reps=30):
    """conv1 on uint8 stacks (k_conv1_u8_bf16x3: bf16 MFMA, weights split into three exact
    bf16 terms) over the learner's 2B stacks of a batch slot, timed alone with HIP events
    around direct launches on the current stream"""
    from reth_amd import _lib
    from reth_amd.fused_learner import _pair
    from reth_amd.replay import FrameStacks

    net = ax.solver.q_network
    frames = isinstance(slot_cols[0], FrameStacks)  # frames in place: conv1 reads the store by frame ids
    x = (FrameStacks.pair if frames else _pair)(slot_cols[0], slot_cols[3])
    n = x.shape[0]
    shape = net._torso_shapes(tuple(x.shape[1:]), True)[0][1]
    pk = net._packed_for(net.pack_convs(), 0, True)
    ho = (shape.hin - shape.kh) // shape.stride + 1
    y = torch.empty((n, shape.cout, ho, ho), device=x.device, memory_format=torch.channels_last)
    bias = net._convs()[0].bias
    ev = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if frames:
            _lib.call("rth_conv1_frames_bias_relu", _lib.ctypes.byref(shape), x.store.data_ptr(), x.ids.data_ptr(), n,
                      pk.data_ptr(), bias.data_ptr(), y.data_ptr(), _lib.stream_ptr())
        else:
            _lib.call("rth_conv_bias_relu", _lib.ctypes.byref(shape), x.data_ptr(), None, n, pk.data_ptr(),
                      bias.data_ptr(), y.data_ptr(), _lib.stream_ptr())
        e1.record()
        ev.append((e0, e1))
    torch.cuda.synchronize()
    t = float(np.median([a.elapsed_time(b) for a, b in ev[5:]])) / 1e3
    flops = 2.0 * n * ho * ho * shape.cout * shape.cin * shape.kh * shape.kw
    src = "frames in place, by frame ids" if frames else "uint8 stacks"
    return {"kernel": f"k_conv1_u8_share ({src}, {n} samples = the learner's [s0; s1])",
            "bound": "mfma", "achieved": round(3 * flops / t / 1e12, 2), "peak": BF16_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(3 * flops / t / 1e12 / BF16_PEAK_TFLOPS, 4),
            "achieved_fp32_equiv": round(flops / t / 1e12, 2), "flops_per_launch": flops,
            "mfma_flops_per_launch": 3 * flops, "launch_us": round(t * 1e6, 2),
            "note": "timed alone after the timed region (HIP events); achieved counts the bf16 MFMA FLOPs issued "
                    "(3 exact-split products per fp32 product), achieved_fp32_equiv the algorithmic ones"}


def conv_impl(shape, n):
    """(kernel label, MFMA FLOPs issued per algorithmic FLOP, peak TFLOP/s of that MFMA) of the
    kernel rth_conv_bias_relu runs for `shape` and n samples (rth_conv_impl)"""
    from reth_amd import _lib

    ns = _lib.ctypes.c_int32(0)
    kind = _lib.lib().rth_conv_impl(_lib.ctypes.byref(shape), int(n), _lib.ctypes.byref(ns))
    if kind == _lib.CONV_IMPL_X9:
        return (f"k_conv_x9 (exact 3 x 3-term bf16 split of input and weights, nine bf16 MFMAs per fp32 product, "
                f"{ns.value} samples per workgroup)", 9, BF16_PEAK_TFLOPS)
    if kind == _lib.CONV_IMPL_BF16X3:
        return "k_conv1_u8_bf16x3 (exact 3-term bf16 split of the weights)", 3, BF16_PEAK_TFLOPS
    return "k_conv_bias_relu (fp32 MFMA)", 1, FP32_PEAK_TFLOPS


def conv_iteration_alone(ax, sizes, reps=20):
    """conv2 / conv3 forward timed alone (HIP events around direct launches, median) at each
    batch size one iteration launches them with ({learner [s0; s1], target pass, actors}):
    the per-iteration kernel time that says which conv kernel dominates the step"""
    from reth_amd import _lib

    net = ax.solver.q_network
    shapes = [sh for _, sh in net._torso_shapes((4, 84, 84), True)]
    packed = net.pack_convs(True)
    out = {}
    for li in (1, 2):
        shape, conv = shapes[li], net._convs()[li]
        ho = (shape.hin - shape.kh) // shape.stride + 1
        per = {}
        for n in sizes:
            x = torch.rand((n, shape.cin, shape.hin, shape.win), device=conv.weight.device).contiguous(
                memory_format=torch.channels_last)
            y = torch.empty((n, shape.cout, ho, ho), device=x.device, memory_format=torch.channels_last)
            ev = []
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                _lib.call("rth_conv_bias_relu", _lib.ctypes.byref(shape), x.data_ptr(), None, n,
                          net._packed_for(packed, li, True).data_ptr(), conv.bias.data_ptr(), y.data_ptr(),
                          _lib.stream_ptr())
                e1.record()
                ev.append((e0, e1))
            torch.cuda.synchronize()
            per[str(n)] = round(float(np.median([a.elapsed_time(b) for a, b in ev[3:]])) * 1e3, 2)
        out[f"conv{li + 1}"] = {"launch_us_by_samples": per, "iteration_us": round(sum(per.values()), 2)}
    return out


def traffic_signature(world, cfg, frame_ids):
    """the run configuration a PMC pass's per-launch byte counts belong to: they are quoted in a
    bench line only when the line's own run has the same signature (a launch's bytes depend on
    the batch, the actors, the replay form and the world size)"""
    return {"world": int(world), "num_actions": int(cfg.num_actions), "batch_size": int(cfg.batch_size),
            "n_actors": int(cfg.n_actors), "capacity": int(cfg.capacity), "frame_store": bool(cfg.frame_store),
            "frame_ids": bool(frame_ids), "env": cfg.env, "actor_steps_per_update": int(cfg.actor_steps_per_update)}


def load_traffic_file(tag, signature):
    """the committed PMC summary of a tagged rocprofv3 pass (scripts/summarize_profile.py TAG:
    separate --pmc FETCH_SIZE / WRITE_SIZE runs, gfx950-corrected) -> (dict, source, reason).
    dict is {} -- every traffic field of the line null -- when the file is absent, records no
    `measured_on`, or was measured on a different configuration than `signature`; reason says
    which."""
    p = os.path.join("profiles", f"traffic_{tag}.json")
    full = os.path.join(ROOT, p)
    if not os.path.exists(full):
        return {}, None, f"no PMC pass {p}"
    with open(full) as f:
        prof = json.load(f)
    on = prof.get("measured_on")
    if on is None:
        return {}, p, f"{p} does not record the configuration it was measured on"
    diff = sorted(k for k in set(on) | set(signature) if on.get(k) != signature.get(k))
    if diff:
        return {}, p, (f"{p} was measured on a different configuration ("
                       + ", ".join(f"{k} {on.get(k)!r} vs {signature.get(k)!r} here" for k in diff) + ")")
    return prof, p, None


def traffic_field(prof, src, reason, key):
    """(bytes or None, source, null_reason) of one traffic field"""
    v = prof.get(key)
    if v is None:
        return None, None, reason or (f"{src} has no {key}" if src else "no PMC pass")
    return v, src, None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


# ----------------------------------------------------------------------------- CPU baseline
def usable_cores():
    """(cores this job may run on, affinity count, cgroup quota in CPUs or None): the affinity
    set capped by the cgroup's cpu.max quota (the GPU box grants a share of a larger host)"""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    use = aff if quota is None else max(1, min(aff, int(quota)))
    return use, aff, quota


def cpu_actor_worker(seconds, idx=None):
    """one reference Ape-X actor process on one core (test/apex-dqn/worker.py:21-61 with
    OMP_NUM_THREADS=1, :3): per env step RandomExploration.act (a batch-1 forward of the host
    solver unless exploring; reth/reth/utils/exploration.py:26-31), a synthetic Pong frame (ALE is
    absent), the f4/i8 casts, NStepAdder.push; per 64 rows calc_loss on the actor's copy
    (dqn_solver.py:100-102) and Client.append's per-row serialize (client.py:27-35; the lz4 and
    the ZMQ send are not included).  Prints env steps/s."""
    torch.set_num_threads(1)
    from reth_amd import pack
    from reth_amd.host_buffer import HostNumpyBuffer
    from reth_amd.nstep import NStepAdder
    from reth_amd.solver import Box, DQNSolver, Discrete

    idx = int(os.environ.get("RTH_CPU_ACTOR_IDX", "0")) if idx is None else idx
    rng = np.random.default_rng(idx)
    torch.manual_seed(0)
    solver = DQNSolver(Box(0, 255, (4, 84, 84)), Discrete(6), gamma=0.99, clip_value=40, double_q=True, dueling=True,
                       learning_rate=1e-4, adam_epsilon=1.5e-4, update_target_interval=100, device="cpu", n_step=3)
    eps = 0.4 ** (1 + (idx % 256) / 255 * 7)
    adder = NStepAdder(0.99, 3)
    buf = HostNumpyBuffer(64, circular=False)
    s0 = rng.integers(0, 256, (4, 84, 84), dtype=np.uint8)
    steps, t0 = 0, time.perf_counter()
    while True:
        if rng.random() < eps:
            a = int(rng.integers(0, 6))
        else:
            a = solver.act(s0)
        s1 = np.concatenate([s0[1:], rng.integers(0, 256, (1, 84, 84), dtype=np.uint8)])
        r, done = float(rng.random() < 0.02), bool(rng.random() < 1 / 2000)
        row = adder.push(np.asarray(s0, dtype="f4"), np.asarray(a, dtype="i8"), np.asarray(r, dtype="f4"),
                         np.asarray(s1, dtype="f4"), np.asarray(done, dtype="f4"))
        s0 = s1
        steps += 1
        if row is not None:
            buf.append(row)
            if buf.size == buf.capacity:
                loss = np.asarray(solver.calc_loss(buf.data), dtype="f4")
                data = buf.data
                rows = [pack.serialize([c[i, ...] for c in data]) for i in range(buf.size)]
                pack.serialize([rows, loss])
                buf.clear()
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    print(json.dumps({"env_steps_per_sec": steps / dt, "steps": steps, "seconds": dt}), flush=True)


def cpu_actor_baseline(procs, seconds=8.0):
    """the reference's actor layout on the host: `procs` single-threaded actor processes
    (cpu_actor_worker), started as child interpreters, run concurrently; aggregate env
    steps/s"""
    import subprocess

    env = dict(os.environ, OMP_NUM_THREADS="1", MKL_NUM_THREADS="1")
    kids = []
    for i in range(procs):
        e = dict(env, RTH_CPU_ACTOR_IDX=str(i * max(1, 256 // procs)))
        kids.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-actor-worker", str(seconds)],
                                     env=e, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True))
    rates = []
    for k in kids:
        out, _ = k.communicate(timeout=seconds + 120)
        for line in out.splitlines():
            if line.startswith("{"):
                rates.append(json.loads(line)["env_steps_per_sec"])
    return {"value": round(float(np.sum(rates)), 1), "unit": "env-steps/s", "cores": procs, "kind": "port",
            "processes_reporting": len(rates), "per_process_env_steps_per_sec": round(float(np.mean(rates)), 1)
            if rates else None,
            "sample": f"{procs} actor processes x {seconds:.0f} s, each the reference worker loop "
                      "(test/apex-dqn/worker.py:37-61) at OMP_NUM_THREADS=1: batch-1 act on the host solver, "
                      "NStepAdder, calc_loss + per-row serialize every 64 rows; synthetic env, no lz4 / ZMQ"}


def cpu_baseline(n_actors=256, batch=512, capacity=1_000_000, ring=20000, iters=6, seed=0):
    """The same Ape-X step on the host: torch-CPU Q-net (all host threads the job owns),
    the oracle's C restatement for tree / PER / n-step / eps-greedy, numpy for the env and
    row storage.  The sum-tree has the full capacity (1 M slots, depth 20); only the frame
    storage is a reduced ring of `ring` rows (slot % ring: host RAM and fill time); the
    per-step work is the full configuration (256 actors, B = 512)."""
    from oracle import oracle as orc
    from reth_amd.model import DQNNetwork

    use, aff, quota = usable_cores()
    torch.set_num_threads(use)
    cores = torch.get_num_threads()
    rng = np.random.default_rng(seed)
    torch.manual_seed(seed)
    qn, tq, an = (DQNNetwork((4, 84, 84), 6) for _ in range(3))
    tq.load_state_dict(qn.state_dict())
    an.load_state_dict(qn.state_dict())
    opt = torch.optim.Adam(qn.parameters(), lr=1e-4, eps=1.5e-4)
    s0s = rng.integers(0, 256, (ring, 4, 84, 84), dtype=np.uint8)
    s1s = rng.integers(0, 256, (ring, 4, 84, 84), dtype=np.uint8)
    acol = rng.integers(0, 6, ring)
    rcol = np.zeros(ring, np.float32)
    dcol = np.zeros(ring, np.float32)
    tree = orc.Tree(capacity)
    tree.update(np.arange(capacity), orc.per_normalize(1.0 - rng.random(capacity, dtype=np.float32), 0.5)
                .astype(np.float64))
    tail = 0
    obs = rng.integers(0, 256, (n_actors, 4, 84, 84), dtype=np.uint8)
    eps = 0.4 ** (1 + np.arange(n_actors) / (n_actors - 1) * 7)
    frames = {}  # handle -> stack (the reference's rows reference frames, never copy them)
    n_handles = n_actors
    obs_h = np.arange(n_actors, dtype=np.int64)
    adders = [orc.NStep(3, 0.99, 0) for _ in range(n_actors)]
    gamma_n = np.float32(0.99 ** 3)

    def step(t):
        nonlocal tail, obs, n_handles
        with torch.no_grad():
            q = an(torch.from_numpy(obs).float()).numpy()
        act = orc.eps_greedy(q, eps, rng.random(n_actors), rng.integers(0, 6, n_actors))
        new = rng.integers(0, 256, (n_actors, 1, 84, 84), dtype=np.uint8)
        nxt = np.concatenate([obs[:, 1:], new], 1)
        r = np.where(rng.random(n_actors) < 0.02, 1.0, 0.0).astype(np.float32)
        d = (rng.random(n_actors) < 1 / 2000).astype(np.float32)
        rows = []
        for i in range(n_actors):
            frames[obs_h[i]] = obs[i]
            h1 = n_handles
            n_handles += 1
            frames[h1] = nxt[i]
            row = adders[i].push(obs_h[i], act[i], r[i], h1, d[i])
            obs_h[i] = h1
            if row is not None:
                rows.append(row)
        obs = nxt
        if rows:  # calc_loss on the actor copy (target == online) + Client.append
            s0 = np.stack([frames[x[0]] for x in rows])
            s1 = np.stack([frames[x[3]] for x in rows])
            for h in [k for k in frames if k < n_handles - 6 * n_actors]:
                del frames[h]
            with torch.no_grad():
                qq = an(torch.from_numpy(np.concatenate([s0, s1])).float()).numpy()
            n = len(rows)
            a_ = np.array([x[1] for x in rows])
            r_ = np.array([x[2] for x in rows], np.float32)
            d_ = np.array([x[4] for x in rows], np.float32)
            td = orc.td_error(qq[:n], qq[n:], qq[n:], a_, r_, d_, gamma_n)
            slots, tail = orc.fifo_indices(capacity, tail, n)
            rs = slots % ring
            s0s[rs], s1s[rs], acol[rs], rcol[rs], dcol[rs] = s0, s1, a_, r_, d_
            tree.update(slots, orc.per_normalize(np.abs(td), 0.5).astype(np.float64))
        # learner update (DQNSolver.update on the CPU)
        idx, p = tree.sample(rng.random(batch))
        isw = orc.per_is_weights(p, tree.min(), 0.4)
        ri = idx % ring
        b0 = torch.from_numpy(s0s[ri]).float()
        b1 = torch.from_numpy(s1s[ri]).float()
        qv = qn(b0)
        with torch.no_grad():
            nt = tq(b1)
            no = qn(b1)
        a_t = torch.from_numpy(acol[ri])
        tdt = qv.gather(1, a_t[:, None])[:, 0] - (torch.from_numpy(rcol[ri]) + float(gamma_n) *
                                                  nt.gather(1, no.argmax(1, keepdim=True))[:, 0] *
                                                  (1 - torch.from_numpy(dcol[ri])))
        loss = (torch.nn.functional.smooth_l1_loss(tdt, torch.zeros_like(tdt), reduction="none") *
                torch.from_numpy(isw).float()).mean()
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(qn.parameters(), 40)
        opt.step()
        tree.update(idx, orc.per_normalize(tdt.detach().abs().numpy(), 0.5).astype(np.float64))

    for t in range(4):  # warm the n-step deques (rows flow from step 4 on)
        step(t)
    t0 = time.perf_counter()
    for t in range(4, 4 + iters):
        step(t)
    dt = time.perf_counter() - t0
    return {"value": round(n_actors * iters / dt, 2), "unit": "env-steps/s", "cores": cores, "kind": "port",
            "affinity_cores": aff, "cgroup_cpu_quota": quota,
            "updates_per_sec": round(iters / dt, 3), "cpu_model": cpu_model(),
            "sample": f"{iters} Ape-X steps (256 actors x 1 env step + 1 B=512 update each), sum-tree of "
                      f"{capacity} slots (depth {int(np.ceil(np.log2(capacity + 1)))}), frame storage a ring of "
                      f"{ring} rows on the host, torch-CPU Q-net + oracle C tree/PER/n-step, "
                      f"{torch.get_num_threads()} threads, {dt:.1f} s"}


# ----------------------------------------------------------------------------- HBM kernels
class ReplayKernelTimer:
    """live in-loop durations of the replay shard's launches (rth_replay_set_timing): before
    every iteration a fresh pair of HIP events per kind is armed; the library records them on
    the launch stream around the next launch of that kind (the append's row copy and tree
    update, the PER sample, the gather)"""
    KINDS = ("tree_update", "sample", "gather", "insert")

    def __init__(self, replay):
        self.h = replay._h
        self.pairs = {k: [] for k in self.KINDS}
        self._armed = None

    def arm(self):
        from reth_amd import _lib

        fired = _lib.c_i32(0)
        evs, cur = [], []
        for _ in self.KINDS:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()  # materialise the events; the library re-records them at the launch
            b.record()
            evs += [a.cuda_event, b.cuda_event]
            cur.append((a, b))
        _lib.call("rth_replay_set_timing", self.h, (_lib.c_vp * len(evs))(*evs), len(evs), _lib.ctypes.byref(fired))
        self._collect(fired.value)
        self._armed = cur

    def stop(self):
        from reth_amd import _lib

        fired = _lib.c_i32(0)
        _lib.call("rth_replay_set_timing", self.h, None, 0, _lib.ctypes.byref(fired))
        self._collect(fired.value)
        self._armed = None

    def _collect(self, mask):
        if self._armed is None:
            return
        for k, (name, pair) in enumerate(zip(self.KINDS, self._armed)):
            if (mask >> (2 * k)) & 3 == 3:
                self.pairs[name].append(pair)

    def mean_us(self, name):
        v = [a.elapsed_time(b) * 1e3 for a, b in self.pairs[name]]
        return (float(np.mean(v)), len(v)) if v else (None, 0)


def hbm_bytes(cfg, n_rows_per_append):
    """algorithmic HBM bytes per launch of the HBM-bound kernels (DESIGN.md 'Kernels'):
    each byte the operation must move once, at the data's storage width"""
    D = int(np.ceil(np.log2(cfg.capacity + 1)))  # tree depth (20 at 1 M)
    B, N, A1 = cfg.batch_size, n_rows_per_append, cfg.num_actions + 1
    keys = N + B  # the append's priorities + the deferred update_priorities of the last update
    row = 2 * STACK + 8 + 4 + 4  # s0, s1 uint8 stacks + a, r, done
    return {
        # per key: the D-level path, each level one 64-B children-pair read + one 32-B node write
        # (the 32-B {sum, val, min} record layout), + the key's index and priority
        "k_tree_update_sub": keys * (D * 96 + 16),
        # per target: D levels x (the left child's sum + the node's value, 16 B) + the leaf's
        # priority, the index and the IS weight written
        "k_tree_sample": B * (D * 16 + 8 + 8 + 8),
        # read + write of every sampled row (uint8 stacks, the HIP torso reads them as they are)
        # + the 5 index reads
        "k_copy_rows (gather)": B * (gather_bytes_per_row(True, True) if cfg.frame_store and cfg.frame_ids and
                                     cfg.hip_conv and cfg.channels_last else
                                     2 * row + 5 * 8 + (2 * 4 * 4 if cfg.frame_store else 0)),
        # the append's rows: each column row read from the actors' ring and written to its slot
        # (frame store: the two stacks' frame ids instead of the stacks)
        "k_copy_rows (insert)": N * (2 * ((2 * 4 * 4 + 16) if cfg.frame_store else row) + 5 * 8),
        # per actor: the FrameStack shift (3 frames read, 4 written) + reward / done / handles /
        # n-step state (~160 B)
        "k_actor_tail": cfg.n_actors * (7 * 84 * 84 + 160),
        # the 3 x B heads rows + a / r / done / isw, |td| out, h1 [B, 2H] read, gh written
        "k_td_heads_backward": B * (3 * A1 * 4 + 8 + 4 + 4 + 8 + 4) + B * 512 * 8,
    }


def hbm_rooflines(ax, timer, probe_ms, tprof, tsrc, treason):
    """roofline_hbm: the HBM-bound kernels north_star names (tree insert / sample / priority
    update, n-step + env (k_actor_tail), TD, gather, clip+Adam) -- algorithmic bytes per launch /
    in-loop launch duration, every duration measured live in the probe window: HIP events
    around the replay's eager launches (rth_replay_set_timing) and around the launches the
    probe graph copies issue between their parts (the actor tail on the actor stream, the
    TD/heads backward and rth_clip_adam on the learner stream).  `traffic` (HBM bytes per
    launch) is PMC data from a separate rocprofv3 pass of the same command, read from
    profiles/traffic_TAG.json and labelled as such -- null (with the reason) when that pass ran
    another configuration (load_traffic_file)."""
    cfg = ax.cfg
    nparams = sum(p.numel() for p in ax.solver._params)
    rows = cfg.n_actors  # one append of N rows per actor step (fused actor: the previous step's rows)
    by = hbm_bytes(cfg, rows)
    # one rank: the norm partials come from conv1's weight-gradient reduce launch (fused_learner
    # NORM_IN_BACKWARD), the step is rth_adam_prenormed = k_adam (reads p, g, m, v; writes p, m, v):
    # 28 B per fp32 parameter; with a gradient all-reduce: rth_clip_adam = k_grad_sqsum (reads g)
    # + k_adam, 32 B
    if getattr(ax.solver, "grad_hook", None) is None:
        clip_name = "rth_adam_prenormed (k_adam)"
        by[clip_name] = nparams * 28
    else:
        clip_name = "rth_clip_adam (k_grad_sqsum + k_adam)"
        by[clip_name] = nparams * 32
    live = {"k_tree_update_sub": "tree_update", "k_tree_sample": "sample", "k_copy_rows (gather)": "gather",
            "k_copy_rows (insert)": "insert"}
    probed = {"k_actor_tail": "actor_tail", "k_td_heads_backward": "td_heads_backward", clip_name: "clip_adam"}
    hbm = tprof.get("hbm_bytes_per_launch", {})
    out = []
    for name, nbytes in by.items():
        us, n, src = None, 0, None
        if name in live:
            us, n = timer.mean_us(live[name])
            src = f"live HIP events (rth_replay_set_timing) in the probe window, {n} launches"
        elif probe_ms.get(probed[name]):
            ms = probe_ms[probed[name]]
            us, n = float(np.mean(ms)) * 1e3, len(ms)
            src = f"live HIP events around the probe graphs' eager launch in the probe window, {n} launches"
        traffic = hbm.get(name)
        ent = {"kernel": name, "bound": "hbm", "bytes_per_launch": int(nbytes), "mean_launch_us": None,
               "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None, "traffic": traffic,
               "traffic_ratio": round(traffic / nbytes, 3) if traffic else None, "time_source": src,
               "traffic_source": f"{tsrc} (PMC pass)" if traffic else None}
        if not traffic:
            ent["traffic_null_reason"] = treason or f"{tsrc} has no entry for {name}"
        if us:
            gbs = nbytes / (us * 1e-6) / 1e9
            ent.update(mean_launch_us=round(us, 2), achieved=round(gbs, 1), frac=round(gbs / HBM_PEAK_GBS, 4))
        out.append(ent)
    return out


# ----------------------------------------------------------------------------- decoupled actors
def decoupled_actors(ax, dev, world, iters=40, sweep=(1, 4, 16)):
    """after the timed region: (1) the actor block alone, learner idle -- the vectorised
    actors' own capacity (env steps + n-step + priorities + appends); (2) the coupled loop at
    actor_steps_per_update in `sweep`.  Ape-X decouples actors from the learner (the reference's
    workers never wait for the trainer), so the headline's fixed 1:1 pairing of one actor step
    per update is a choice of replay ratio; these say what other ratios give.  Every rank runs
    the same iterations (the learner all-reduces); times are max over ranks."""
    import torch.distributed as dist

    def timed(fn, n):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t)
        return dt

    keep = ax.cfg.actor_steps_per_update
    out = {}
    ax.cfg.actor_steps_per_update = 1
    for _ in range(3):  # each synchronized: no host backlog into timed()'s first sync (main(), settle)
        ax.actor_iteration()
        torch.cuda.synchronize()
    e0 = ax.env_steps
    dt = timed(ax.actor_iteration, iters)
    out["actor_only_env_steps_per_sec"] = round((ax.env_steps - e0) * world / dt, 1)
    out["actor_only_ms_per_actor_step"] = round(dt / iters * 1e3, 4)
    out["sweep"] = []
    for k in sweep:
        ax.cfg.actor_steps_per_update = k
        for _ in range(2):
            ax.iteration()
            torch.cuda.synchronize()
        u0, e0 = ax.updates, ax.env_steps
        n = max(4, iters // k)
        dt = timed(ax.iteration, n)
        out["sweep"].append({"actor_steps_per_update": k, "env_steps_per_sec": round((ax.env_steps - e0) * world / dt, 1),
                             "learner_updates_per_sec": round((ax.updates - u0) * world / dt, 2),
                             "ms_per_step": round(dt / n * 1e3, 4)})
    ax.cfg.actor_steps_per_update = keep
    out["note"] = ("measured after the timed region on the same process: actor_only = the captured actor block "
                   "replayed with the learner stream idle; sweep = the coupled loop at other actor:learner ratios "
                   "(the headline runs actor_steps_per_update = config.actor_steps_per_update)")
    return out


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="pong",
                    help="pong (= pong-node) = BASELINE configs[1] at N = 1, configs[3] at N > 1 (256 actors and "
                         "1 M rows sharded over the N GPUs); pong-weak = configs[1] on every GPU; breakout = "
                         "configs[2] (2048 actors, 4 M replay, A = 4: 225.9 GB of full-row uint8 storage)")
    ap.add_argument("--actors", type=int, default=None)
    ap.add_argument("--capacity", type=int, default=None)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--faithful", action="store_true",
                    help="SURVEY §8(d) C4 hyperparameter-faithful data parallelism: a global batch of --batch "
                         "split over the N learners (B / N per GPU) instead of B per GPU")
    ap.add_argument("--windows", type=int, default=5, help="sub-windows of the timed region reported beside it")
    ap.add_argument("--settle", type=int, default=256, help="iterations of the captured loop between the graph "
                    "capture and the W warmup steps (setup, not timed)")
    ap.add_argument("--probe-steps", type=int, default=60, help="iterations of the probe window after the timed "
                    "region (live per-launch HIP-event timing of the roofline kernels)")
    ap.add_argument("--no-probe", action="store_true", help="do not cut the learner graph around conv2/conv3 "
                    "(no live per-launch timing of the dominant kernels)")
    ap.add_argument("--actor-steps-per-update", type=int, default=None,
                    help="vectorised actor steps per learner update (default 1; N for the sharded pong workload)")
    ap.add_argument("--env", choices=["synthetic", "atari", "atari-h2d"], default="synthetic",
                    help="actors' observations: synthetic uint8 stacks (default); atari = raw 210x160 RGB frame pairs "
                         "from device Philox through the device MaxAndSkip / gray / INTER_AREA / FrameStack; atari-h2d = "
                         "the same with the raw pairs copied host -> device from pinned memory every step (host ALE)")
    ap.add_argument("--frame-store", action="store_true", default=True,
                    help="frame de-duplicated replay (SURVEY §8(d) C3; the default since r04): each actor frame "
                         "stored once in an HBM frame store, rows keep their stacks as frame ids, the gather "
                         "copies the ids and conv1 reads the frames in place (RTH_FRAME_IDS=0: the gather assembles "
                         "the stacks) -- bit-identical rows and updates (tests/test_frame_store_gpu.py), Pong's 1 M "
                         "rows in 14.1 GB instead of 56.5 (hard bound), Breakout's 4 M in 56.7 instead of 225.9, and no "
                         "56 KB stack copies per inserted row (Pong 0.563-0.564 vs 0.571-0.574 ms/step interleaved)")
    ap.add_argument("--frame-store-bound", choices=["hard", "expected"], default="hard",
                    help="frame store size: hard = the worst case (2 frames per actor step: no live row's frames are "
                         "ever overwritten); expected = sized for the i.i.d. episode-end rate (half the bytes)")
    ap.add_argument("--full-rows", dest="frame_store", action="store_false",
                    help="store both uint8 stacks of every row, as the reference's worker does (worker.py:44-51)")
    ap.add_argument("--no-sweep", action="store_true", help="skip the decoupled-actor measurements after the "
                    "timed region (actor block alone; actor_steps_per_update 1 / 4 / 16)")
    ap.add_argument("--cpu-actor-worker", type=float, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-iters", type=int, default=72)
    ap.add_argument("--tag", default="r06", help="profiles/traffic_TAG.json: the PMC pass the traffic fields cite")
    ap.add_argument("--nchw", action="store_true", help="contiguous NCHW Q-net tensors (default channels-last)")
    ap.add_argument("--no-conv-benchmark", action="store_true", help="MIOpen immediate mode instead of find")
    ap.add_argument("--eager", action="store_true", help="no HIP-graph replay (launch every kernel from Python)")
    ap.add_argument("--wgrad", choices=["miopen", "f32", "x9"], default=None,
                    help="conv2 / conv3 weight gradients (default: fused_learner.HIP_WGRAD)")
    ap.add_argument("--no-fc1-heads", action="store_true",
                    help="FC1's reduce and FC2 as two launches (model.FC1_HEADS off; A/B aid)")
    ap.add_argument("--miopen-conv", action="store_true", help="conv torso forward in MIOpen (+ rth_bias_relu) "
                    "instead of rth_conv_bias_relu")
    args = ap.parse_args()
    if args.cpu_actor_worker is not None:  # a child of cpu_actor_baseline (never touches the GPU)
        return cpu_actor_worker(args.cpu_actor_worker)
    wl = WORKLOADS[args.workload]
    shard = wl["shard"] and args.gpus > 1
    if shard and (wl["actors"] % args.gpus or wl["capacity"] % args.gpus):
        raise SystemExit(f"--workload {args.workload}: {wl['actors']} actors / {wl['capacity']} rows do not split "
                         f"over {args.gpus} GPUs")
    args.actors = (wl["actors"] // args.gpus if shard else wl["actors"]) if args.actors is None else args.actors
    args.capacity = (wl["capacity"] // args.gpus if shard else wl["capacity"]) if args.capacity is None else args.capacity
    if args.actor_steps_per_update is None:
        args.actor_steps_per_update = args.gpus if shard else 1

    from reth_amd.apex import ApexConfig, ApexDQN
    from reth_amd.dist import init_from_env, shutdown

    if os.environ.get("RTH_CUDNN_DET") == "1":  # A/B aid: MIOpen's deterministic solvers (no atomic wrw + fills)
        torch.backends.cudnn.deterministic = True
    if os.environ.get("RTH_BLAS"):  # A/B aid: torch's GEMM backend ("cublas" = rocBLAS, "cublaslt" = hipBLASLt)
        torch.backends.cuda.preferred_blas_library(os.environ["RTH_BLAS"])

    import torch.distributed as dist

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("RTH_SHARE_GPU"):  # rehearsal of N ranks on fewer GPUs (with RTH_DIST_BACKEND=gloo)
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    rank, world = init_from_env()
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but the process group has {world} rank(s) "
                         f"(WORLD_SIZE={world_env}): launch N > 1 under torch.distributed.run")
    backend = dist.get_backend() if world > 1 else None
    if world > 1 and rank == 0:
        print(f"data-parallel learner: {world} ranks over {backend} "
              f"({'RCCL' if backend == 'nccl' else backend}), one GPU each", file=sys.stderr, flush=True)
    dev = torch.device("cuda", local)
    per_gpu_batch = args.batch
    if args.faithful:
        if args.batch % world:
            raise SystemExit(f"--faithful: global batch {args.batch} does not split over {world} GPUs")
        per_gpu_batch = args.batch // world
    if args.no_fc1_heads:
        from reth_amd import model
        model.FC1_HEADS = False
    if args.wgrad is not None:
        from reth_amd import fused_learner
        fused_learner.HIP_WGRAD = None if args.wgrad == "miopen" else args.wgrad
    hip_conv = not args.miopen_conv
    probe = hip_conv and not args.nchw and not args.eager and not args.no_probe
    cfg = ApexConfig(n_actors=args.actors, capacity=args.capacity, batch_size=per_gpu_batch, num_actions=wl["actions"],
                     actor_steps_per_update=args.actor_steps_per_update, seed=0,
                     channels_last=not args.nchw, conv_benchmark=not args.no_conv_benchmark,
                     hip_graph=not args.eager, hip_conv=hip_conv, env=args.env, frame_store=args.frame_store,
                     frame_store_bound=args.frame_store_bound,
                     frame_ids=args.frame_store and os.environ.get("RTH_FRAME_IDS", "1") == "1", extra={"learner_priority": int(os.environ.get("RTH_LEARNER_PRIORITY", "0")),
                            "actor_priority": int(os.environ.get("RTH_ACTOR_PRIORITY", "0")),
                            "probe_conv2": probe})
    ax = ApexDQN(cfg, device=dev, rank=rank, world=world)
    ax.prefill(cfg.capacity)
    # graph preparation (setup, like the prefill): iterate until the actor / learner / target
    # graphs are captured, upload every captured graph (hipGraphUpload: a variant first replayed
    # inside the timed region -- the learner's "full" variant after a target sync, the actors'
    # "full" pass after a weights reload -- does not pay its first-launch cost there), then
    # `settle` iterations of the captured loop, so the timed region starts in the loop's steady
    # state (r03's driver windows fell 0.663 -> 0.600 ms over the first 20 steps after capture);
    # then the W warmup steps the command asks for
    prep = {"capture_iterations": 0, "settle_iterations": 0, "graphs_uploaded": 0}
    if cfg.hip_graph:
        while ax._graphs is None and prep["capture_iterations"] < 64:
            ax.iteration()
            prep["capture_iterations"] += 1
        if ax._graphs is not None:
            prep["graphs_uploaded"] = ax.upload_graphs()
            # the host must not run far ahead of the GPU into the synchronize before the timed
            # region: after a sync that drained a ~125 ms backlog the first timed step's enqueue
            # took 1.2-1.6 ms instead of 0.1 (r04 probe: 0.643 ms/step over 20 steps, flat
            # 0.581 with the backlog bounded), so the settle iterations synchronize every 8th
            # and each of the last 16, the warmup steps each
            for i in range(args.settle):
                ax.iteration()
                if i % 8 == 7 or i >= args.settle - 16:
                    torch.cuda.synchronize()
            prep["settle_iterations"] = args.settle
    for i in range(args.warmup):
        ax.iteration()
        torch.cuda.synchronize()

    # live per-launch timing (the probe window after the headline): HIP events on the launching
    # stream around the launches the probe graph copies leave out -- conv2 / conv3 forward, the
    # TD/heads backward and clip+Adam on the learner stream, the actor tail on the actor stream
    # (ApexDQN._replay_parts / _learner_replay call conv_probe between the parts) -- and the
    # replay shard's eager launches (ReplayKernelTimer)
    conv_events = {"conv2": [], "conv3": []}

    def conv_probe(tag):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        base = tag[:-len("_end")] if tag.endswith("_end") else tag
        ev = conv_events.setdefault(base, [])
        if base == tag:
            ev.append([e, None])
        elif ev and ev[-1][1] is None:
            ev[-1][1] = e
    spans = []
    if os.environ.get("RTH_BENCH_SPAN"):  # diagnostics: the learner block's span on its stream
        replay = ax._learner_replay

        def timed_replay(v):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            replay(v)
            b.record()
            spans.append((a, b))
        ax._learner_replay = timed_replay
        ready = []  # when each batch's sample + target pass were done on the actor stream

        class _Ready:  # ApexDQN._ev_sample with a timing twin
            def __init__(self, ev):
                self.ev = ev

            def record(self, stream=None):
                self.ev.record(stream)
                t = torch.cuda.Event(enable_timing=True)
                t.record(stream)
                ready.append(t)

            def wait(self, stream=None):
                self.ev.wait(stream)

        ax._ev_sample = _Ready(ax._ev_sample)
    u0, e0 = ax.updates, ax.env_steps
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # ------------------------------------------------------------------ the timed region
    # the uncut graphs, no per-launch timers: sub-window boundaries are events on the iteration
    # stream (no synchronisation inside the timed region); the headline is the whole region
    n_win = max(1, min(args.windows, args.steps))
    win_at = {round(args.steps * i / n_win) for i in range(n_win + 1)}
    win_ev = []
    t0 = time.perf_counter()
    debug = os.environ.get("RTH_BENCH_DEBUG")
    step_ev = [] if os.environ.get("RTH_BENCH_STEPTIMES") else None
    host_ms = []
    for k in range(args.steps):
        if k in win_at:
            e = torch.cuda.Event(enable_timing=True)
            e.record(ax._stream if hasattr(ax, "_stream") else None)
            win_ev.append((k, e))
        if step_ev is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record(ax._stream)
            step_ev.append(e)
        th = time.perf_counter()
        if k == 0 and os.environ.get("RTH_BENCH_PROFILE0"):  # diagnostics: where step 0's host time goes
            import cProfile
            import pstats

            pr = cProfile.Profile()
            pr.runcall(ax.iteration)
            pstats.Stats(pr, stream=sys.stderr).sort_stats("tottime").print_stats(12)
        else:
            ax.iteration()
        if step_ev is not None:
            host_ms.append((time.perf_counter() - th) * 1e3)
        if debug:
            torch.cuda.synchronize()
            print(f"rank {rank} step {k}: {1e3 * (time.perf_counter() - t0):.1f} ms graphs={ax._graphs is not None} "
                  f"updates={ax.updates} pending={ax.loader.pending()}", file=sys.stderr, flush=True)
    e = torch.cuda.Event(enable_timing=True)
    e.record(ax._stream)
    win_ev.append((args.steps, e))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    n_upd, n_env = ax.updates - u0, ax.env_steps - e0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
        c = torch.tensor([n_env, n_upd], dtype=torch.float64, device=dev)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        n_env, n_upd = int(c[0]), int(c[1])
    if spans:
        busy = [a.elapsed_time(b) * 1e3 for a, b in spans]
        gaps = [spans[i][1].elapsed_time(spans[i + 1][0]) * 1e3 for i in range(len(spans) - 1)]
        print(f"learner block span {np.mean(busy):.1f} us (min {np.min(busy):.1f}), gap to the next "
              f"{np.mean(gaps):.1f} us (median {np.median(gaps):.1f}), over {len(busy)} updates", file=sys.stderr)
        if ready:  # actor stream's batch ready vs the learner block's previous end: > 0 = the learner waited
            m = min(len(ready), len(spans) - 1)
            late = [spans[i][1].elapsed_time(ready[i]) * 1e3 for i in range(m)]
            print(f"next batch ready after the learner block ends: mean {np.mean(late):.1f} us, median "
                  f"{np.median(late):.1f}, > 0 in {np.mean(np.array(late) > 0) * 100:.0f} % of updates", file=sys.stderr)
    if step_ev is not None:
        step_ev.append(win_ev[-1][1])
        print("per-step ms: " + " ".join(f"{a.elapsed_time(b):.3f}" for a, b in zip(step_ev, step_ev[1:])),
              file=sys.stderr, flush=True)
        print("host enqueue ms: " + " ".join(f"{h:.3f}" for h in host_ms), file=sys.stderr, flush=True)
    win_ms = [a[1].elapsed_time(b[1]) / (b[0] - a[0]) for a, b in zip(win_ev, win_ev[1:])]
    # ------------------------------------------------------------------ the probe window
    # after the headline: the probe graph copies replay with HIP events around the timed
    # launches, and the replay shard's launches are timed by ReplayKernelTimer
    ktimer = ReplayKernelTimer(ax.replay)
    probe_steps, probe_ms_per_step = 0, None
    if args.probe_steps > 0:
        ax.conv_probe = conv_probe if probe else None
        for _ in range(3):  # the probe copies' first replays (uploaded, but their eager launches are new)
            ax.iteration()
        for v in conv_events.values():
            v.clear()
        tp0 = time.perf_counter()
        for _ in range(args.probe_steps):
            ktimer.arm()
            ax.iteration()
        ktimer.stop()
        torch.cuda.synchronize()
        probe_ms_per_step = (time.perf_counter() - tp0) * 1e3 / max(1, args.probe_steps)
        probe_steps = args.probe_steps
        ax.conv_probe = None
    conv_ms = {t: [a.elapsed_time(b) for a, b in ev if b is not None] for t, ev in conv_events.items()}
    conv2_ms, conv3_ms = conv_ms["conv2"], conv_ms["conv3"]
    replicas = None
    if world > 1:  # the data-parallel replicas must hold identical parameters
        with torch.no_grad():
            hsum = torch.stack([p.double().sum() for p in ax.solver.q_network.parameters()]).sum()
            hsq = torch.stack([p.double().square().sum() for p in ax.solver.q_network.parameters()]).sum()
        mine = torch.stack([hsum, hsq]).to(dev)
        allh = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allh, mine)
        replicas = all(torch.equal(allh[0], h) for h in allh[1:])
    gather_ms = [a.elapsed_time(b) for a, b in ktimer.pairs["gather"]]
    mean_gather_s = float(np.mean(gather_ms)) / 1e3
    fids = bool(cfg.frame_store and cfg.frame_ids and cfg.hip_conv and cfg.channels_last)
    bytes_launch = (gather_bytes_per_row(cfg.hip_conv and cfg.channels_last, fids) +
                    (32 if cfg.frame_store and not fids else 0)) * cfg.batch_size  # frame store: + the ids read
    achieved = bytes_launch / mean_gather_s / 1e9
    # the same gather alone on the GPU (in the timed region it shares the GPU with the
    # concurrently running learner block): context for the in-loop figure, not `achieved`
    slot_cols, slot_idx, _ = ax.loader._slots[0]
    iso = []
    for _ in range(30):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ax.replay.gather(slot_idx, out_cols=slot_cols)
        e1.record()
        iso.append((e0, e1))
    torch.cuda.synchronize()
    iso_s = float(np.median([a.elapsed_time(b) for a, b in iso[5:]])) / 1e3
    conv1 = conv1_roofline(ax, slot_cols) if cfg.hip_conv and cfg.channels_last else None
    conv_alone = conv_iteration_alone(ax, (2 * cfg.batch_size, cfg.batch_size, cfg.n_actors)) \
        if cfg.hip_conv and cfg.channels_last else None
    decoupled = None
    if not args.no_sweep and ax._graphs is not None:
        decoupled = decoupled_actors(ax, dev, world)
    if rank != 0:  # no collective after this point (rank 0 only assembles and prints the line)
        if world > 1:
            shutdown(ax)  # graphs released, then the process group destroyed (reth_amd.dist)
        return
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(n_actors=cfg.n_actors, batch=cfg.batch_size, iters=args.cpu_iters)
        cpu["reference_actor_layout"] = cpu_actor_baseline(usable_cores()[0])
    f = qnet_flops_per_sample(cfg.num_actions)
    flops_update = 5 * cfg.batch_size * f  # online fwd on s0 + s1, target fwd on s1, bwd (~2 fwd)
    # actors: the acting stacks (N) -- the rows' heads come from the per-stack cache
    # (VecActors.step_fused dedup mode; the terminal stacks of ended episodes, ~N/2000 per
    # step, and the full passes after a weights reload are not counted)
    flops_actor = cfg.n_actors * f * args.actor_steps_per_update
    flops_step = flops_update + flops_actor
    step_s = dt / args.steps
    tsig = traffic_signature(world, cfg, fids)
    tprof, tsrc, treason = load_traffic_file(args.tag, tsig)
    traffic, traffic_src, traffic_null = traffic_field(tprof, tsrc, treason, "gather_hbm_bytes_per_launch")
    c2_traffic, c2_src, c2_null = traffic_field(tprof, tsrc, treason, "conv2_learner_hbm_bytes_per_launch")
    c3_traffic, c3_src, c3_null = traffic_field(tprof, tsrc, treason, "conv3_learner_hbm_bytes_per_launch")
    roofline_gather = {
        "kernel": "rth_replay_gather (k_copy_rows: PER-sampled rows, frames %s)"
                  % ("as frame ids (conv1 reads the store)" if fids else
                     "uint8 stacks" if cfg.hip_conv and cfg.channels_last else "u8->f32 NHWC"),
        "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
        "traffic_null_reason": traffic_null, "bytes_per_launch": bytes_launch, "mean_launch_us": round(mean_gather_s * 1e6, 2),
        "launches_timed": len(gather_ms), "isolated_launch_us": round(iso_s * 1e6, 2),
        "isolated_frac": round(bytes_launch / iso_s / 1e9 / HBM_PEAK_GBS, 4),
        "note": "timed in the probe window; the gather overlaps the learner block on a second stream"}
    roofline = roofline_gather
    n2 = 2 * cfg.batch_size  # the learner's [s0; s1] forward

    torso = [sh for _, sh in ax.solver.q_network._torso_shapes((4, 84, 84), True)]

    def conv_roofline(ms, name, cin, hin, cout, hout, k, stride, flops, traffic, src, null_reason):
        s_ = float(np.mean(ms)) / 1e3
        label, issue, unit_peak = conv_impl(torso[int(name[-1]) - 1], n2)
        r = {
            "kernel": f"{name}: {label}; {cin}x{hin}x{hin} -> {cout}x{hout}x{hout}, k{k} s{stride}, in the "
                      f"learner's [s0; s1] forward, {n2} samples per launch",
            "bound": "mfma", "achieved": round(flops / s_ / 1e12, 2), "peak": FP32_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(flops / s_ / 1e12 / FP32_PEAK_TFLOPS, 4),
            "traffic": traffic, "traffic_source": src, "traffic_null_reason": null_reason, "flops_per_launch": flops,
            "algorithmic_bytes_per_launch": n2 * (hin * hin * cin + hout * hout * cout) * 4 + cout * k * k * cin * 4 + cout * 4,
            "mean_launch_us": round(s_ * 1e6, 2), "median_launch_us": round(float(np.median(ms)) * 1e3, 2),
            "launches_timed": len(ms),
            "note": "timed live in the probe window after the timed region: HIP events on the learner stream around "
                    "the launch (the probe copy of the learner graph is cut there); it runs concurrently with the "
                    "actor stream's kernels"}
        if issue > 1:  # exact-split bf16 kernel: achieved / frac are fp32-equivalent (the dtype's peak)
            r["mfma_issue"] = {"bf16_flops_per_launch": issue * flops, "achieved": round(issue * flops / s_ / 1e12, 2),
                               "peak": unit_peak, "frac": round(issue * flops / s_ / 1e12 / unit_peak, 4),
                               "note": f"the bf16 MFMA FLOPs the kernel issues ({issue} exact-split products per fp32 "
                                       "product) against the dense bf16 peak"}
        return r

    roofline_conv2 = None
    if conv2_ms:
        roofline_conv2 = conv_roofline(conv2_ms, "conv2", 32, 20, 64, 9, 4, 2, 2.0 * n2 * 9 * 9 * 64 * 32 * 4 * 4,
                                       c2_traffic, c2_src, c2_null)
        roofline = roofline_conv2
    roofline_conv3 = None
    if conv3_ms:
        roofline_conv3 = conv_roofline(conv3_ms, "conv3", 64, 9, 64, 7, 3, 1, 2.0 * n2 * 7 * 7 * 64 * 64 * 3 * 3,
                                       c3_traffic, c3_src, c3_null)
    # `roofline` = the conv kernel with the most time per iteration (its three launches -- learner,
    # target pass, actors -- timed alone at their batch sizes)
    if roofline_conv2 and roofline_conv3:
        roofline = roofline_conv3 if conv_alone["conv3"]["iteration_us"] >= conv_alone["conv2"]["iteration_us"] \
            else roofline_conv2
    elif roofline_conv3:
        roofline = roofline_conv3
    out = {
        "metric": "env-steps/sec + learner updates/sec, Ape-X DQN Pong, 1/2/4/8 MI355X",
        "value": round(n_env / dt, 1),
        "unit": "env-steps/s",
        "learner_updates_per_sec": round(n_upd / dt, 2),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 3),
        "ms_per_step_windows": [round(w, 4) for w in win_ms],
        "ms_per_step_window_median": round(float(np.median(win_ms)), 4) if win_ms else None,
        "graph_prepare": dict(prep, note="setup before the W warmup steps: the capture iterations, hipGraphUpload of "
                                         "every captured graph, then `settle` untimed iterations of the captured loop "
                                         "(synchronized every 8th and the last 16; each warmup step synchronized: the "
                                         "host never enters the timed region's first sync far ahead of the GPU)"),
        "probe_window": {"steps": probe_steps, "ms_per_step": round(probe_ms_per_step, 4) if probe_ms_per_step else None,
                         "note": "after the timed region: the probe graph copies (cut at the timed launches) + the "
                                 "replay shard's launch timers; every per-launch time in this line comes from it"},
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": ("synthetic (Philox uint8 Pong-shaped frames, random-init Q-net; no ALE/checkpoints on the box)"
                 if args.env == "synthetic" else
                 "synthetic raw 210x160x3 screens (Philox%s) through the device Atari preprocessing, random-init Q-net; "
                 "no ALE/checkpoints on the box" % (", copied host -> device from pinned memory every step"
                                                     if args.env == "atari-h2d" else " on the device")),
        "config": {"workload": (wl["name_node"].format(n=world) if shard else wl["name"]),
                   "baseline_config": ("configs[3]" if shard else {"pong": "configs[1]", "pong-node": "configs[1]",
                                                                   "pong-weak": "configs[1]" if world == 1 else
                                                                   "configs[1] x N (weak)",
                                                                   "breakout": "configs[2]"}[args.workload]),
                   "actors_per_gpu": cfg.n_actors, "actors_total": cfg.n_actors * world,
                   "replay_capacity_total": cfg.capacity * world, "num_actions": cfg.num_actions,
                   "replay_capacity_per_gpu": cfg.capacity, "replay_prefilled": True, "batch_size": cfg.batch_size,
                   "n_step": cfg.n_step, "alpha": cfg.alpha, "beta": cfg.beta,
                   "actor_steps_per_update": cfg.actor_steps_per_update, "env": cfg.env,
                   "replay_storage": replay_storage(ax),
                   "qnet_layout": "channels_last" if cfg.channels_last else "nchw",
                   "conv_benchmark": cfg.conv_benchmark, "hip_graph": cfg.hip_graph, "hip_conv": cfg.hip_conv,
                   "global_batch": cfg.batch_size * world,
                   "batch_mode": "hyperparameter-faithful (global batch split over the learners)" if args.faithful
                                 else "throughput (B per GPU)",
                   "parallelism": (f"dp{world} learner (RCCL grad all-reduce) + {world} replay shards" if world > 1
                                   else "one GPU: actors, replay shard and learner")},
        "dist": {"world": world, "backend": backend, "rccl": backend == "nccl",
                 "replicas_identical": replicas} if world > 1 else None,
        "roofline": roofline,
        "roofline_gather": roofline_gather,
        "roofline_conv2": roofline_conv2,
        "roofline_conv3": roofline_conv3,
        "conv_iteration_alone": conv_alone,
        "qnet_mfma": {"tflops_per_step": round(flops_step / 1e12, 4),
                      "achieved_tflops": round(flops_step / step_s / 1e12, 2),
                      "peak_fp32_tflops": FP32_PEAK_TFLOPS},
        "roofline_conv1": conv1,
        "roofline_hbm": hbm_rooflines(ax, ktimer, conv_ms, tprof, tsrc, treason),
        "traffic_measured_on": tprof.get("measured_on") if tprof else None,
        "decoupled_actors": decoupled,
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
    if world > 1:
        shutdown(ax)


if __name__ == "__main__":
    main()
