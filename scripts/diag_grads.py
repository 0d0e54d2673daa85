"""Learner gradients on the golden Pong B=512 batch (tests/golden/dqn_pong_b512.npz): the
explicit pass (fused_learner.dueling_grads) run eagerly from the reference's seeded init,
every parameter gradient and |td| dumped to gpurun_out/grads_<tag>.npz.  `--check <npz>...`
(CPU) compares dumps with the float64 gradient of the reference loss (dqn_solver.py:68-117)
on the same init.  Diagnostic only."""
import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

from dqn_batch import apex_batch  # noqa: E402

B, A = 512, 6
SEED = int(np.load(os.path.join(ROOT, "tests", "golden", "dqn_pong_b512.npz"))["seed"])  # the screened seed


def dump(tag):
    from reth_amd.solver import Box, DQNSolver, Discrete

    dev = torch.device("cuda:0")
    torch.manual_seed(SEED)
    solver = DQNSolver(Box(0, 255, (4, 84, 84)), Discrete(A), gamma=0.99, clip_value=40, double_q=True, dueling=True,
                       learning_rate=1e-4, adam_epsilon=1.5e-4, update_target_interval=100, device=dev, n_step=3,
                       channels_last=True)
    s0, s1, a, r, done, isw = apex_batch(SEED, B, A)
    frames = torch.as_tensor(np.concatenate([s0, s1])).to(dev)
    td = solver.compute_grads([frames[:B], a, r, frames[B:], done], weights=torch.as_tensor(isw)).cpu().numpy()
    out = {"td": td}
    for name, p in solver.q_network.named_parameters():
        out[name] = p.grad.detach().double().cpu().numpy()
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez_compressed(f"gpurun_out/grads_{tag}.npz", **out)
    print("dumped", tag, flush=True)


def exact_grads():
    from reth_amd.model import make_q_network

    torch.manual_seed(SEED)
    q = make_q_network((4, 84, 84), A)
    t = make_q_network((4, 84, 84), A)
    t.load_state_dict(q.state_dict())
    q, t = q.double(), t.double()
    s0, s1, a, r, done, isw = apex_batch(SEED, B, A)
    s0, s1 = torch.as_tensor(s0).double(), torch.as_tensor(s1).double()
    a, r, done = torch.as_tensor(a).long(), torch.as_tensor(r).double(), torch.as_tensor(done).double()
    qv = q(s0).gather(1, a.view(-1, 1)).view(-1)
    with torch.no_grad():
        best = q(s1).argmax(1)
        nxt = t(s1).gather(1, best.view(-1, 1)).view(-1)
        target = r + 0.99 ** 3 * nxt * (1 - done)
    td = qv - target
    loss = (F.smooth_l1_loss(td, torch.zeros_like(td), reduction="none") * torch.as_tensor(isw).double()).mean()
    loss.backward()
    return td.detach().abs().numpy(), {n: p.grad.numpy() for n, p in q.named_parameters()}


def check(paths):
    td64, g64 = exact_grads()
    for path in paths:
        d = np.load(path)
        print(path, "|td| max err", np.abs(d["td"] - td64).max())
        for n, g in g64.items():
            e = np.abs(d[n] - g)
            print(f"  {n:20s} max|g| {np.abs(g).max():.2e} max err {e.max():.2e} rel {e.max() / np.abs(g).max():.2e} "
                  f"n(err>1e-3 max|g|) {(e > 1e-3 * np.abs(g).max()).sum()}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="x9")
    ap.add_argument("--check", nargs="*")
    args = ap.parse_args()
    if args.check:
        check(args.check)
    else:
        dump(args.tag)
