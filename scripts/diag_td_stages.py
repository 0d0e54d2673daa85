"""Where the learner's end-to-end |td| error comes from: the
golden Pong batch (dqn_pong_b512: B = 512, A = 6, the reference's seeded init, target = online)
through the learner's forward stage by stage -- conv1, conv2, conv3 (= the FC1 input), FC1
(+ bias + ReLU), the raw heads (FC2), Q(s0, a), the double-Q target and td -- in three arithmetics:

  ours   the HIP path the captured learner runs (rth_conv_bias_relu x3, the FC1 GEMM with its
         bias + ReLU epilogue, rth_heads_fc2, rth_td_huber for td)
  ref32  the reference's own fp32 arithmetic: torch on the CPU, float32 (what
         reth/reth/algorithm/dqn/dqn_solver.py:68-89 computes there)
  exact  the same network in float64 on the CPU

Per stage it prints the max |ours - exact| and |ref32 - exact| over the stage's outputs
("propagated": each path fed its own previous stage), and the error the stage ADDS by itself
("local": every path fed the exact previous stage rounded to fp32), each also relative to the
stage's operand scale sum|x||w|.  Diagnostic only: the assertions live in
tests/test_learner_full_gpu.py.  Writes the table to stdout and, with an argument, as JSON."""
import ctypes
import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

from dqn_batch import apex_batch, frames_sha  # noqa: E402

from reth_amd import _lib  # noqa: E402
from reth_amd.model import fc1_relu, make_q_network, nchw_out  # noqa: E402
from reth_amd.solver import td_huber_forward  # noqa: E402


def combine(heads):
    """dueling combination (dqn_model.py:58-71): Q = V + A - mean(A)"""
    adv, val = heads[:, :-1], heads[:, -1:]
    return val + adv - adv.mean(dim=1, keepdim=True)


def td_of(q0h, q1h_online, q1h_target, a, r, done, gamma_n):
    """double-Q td (dqn_solver.py:68-89) from raw heads, in the heads' own dtype"""
    q0 = combine(q0h).gather(1, a.view(-1, 1)).squeeze(1)
    a1 = combine(q1h_online).argmax(dim=1)
    q1 = combine(q1h_target).gather(1, a1.view(-1, 1)).squeeze(1)
    target = r + gamma_n * (1 - done) * q1
    return q0, target, target - q0


def main():
    dev = torch.device("cuda:0")
    gd = np.load(os.path.join(ROOT, "tests", "golden", "dqn_pong_b512.npz"), allow_pickle=False)
    B, A, seed = int(gd["B"]), int(gd["A"]), int(gd["seed"])
    s0, s1, a, r, done, isw = apex_batch(seed, B, A)
    assert frames_sha(s0, s1) == str(gd["frames_sha"])
    torch.manual_seed(seed)
    net = make_q_network((4, 84, 84), A).to(dev)
    sums = np.array([float(v.double().cpu().contiguous().sum()) for v in net.state_dict().values()])
    assert np.allclose(sums, gd["init_sum"], rtol=1e-10, atol=1e-9), "not the reference's seeded init"
    gamma_n = 0.99 ** 3
    cpu32 = make_q_network((4, 84, 84), A)
    cpu32.load_state_dict({k: v.detach().cpu() for k, v in net.state_dict().items()})
    cpu64 = make_q_network((4, 84, 84), A).double()
    cpu64.load_state_dict({k: v.detach().cpu().double() for k, v in net.state_dict().items()})
    x8 = torch.as_tensor(np.concatenate([s0, s1]))
    n = 2 * B
    a_t, r_t, d_t = torch.as_tensor(a), torch.as_tensor(r), torch.as_tensor(done)

    convs_g = net._convs()
    shapes = [sh for _, sh in net._torso_shapes((4, 84, 84), True)]
    packed = net.pack_convs(True)

    def conv_gpu(li, h):
        shape = shapes[li]
        last = li == len(shapes) - 1
        ho = (shape.hin - shape.kh) // shape.stride + 1
        y = torch.empty((n, shape.cout, ho, ho), dtype=torch.float32, device=dev,
                        memory_format=torch.contiguous_format if last else torch.channels_last)
        hh = h.contiguous() if li == 0 else h.contiguous(memory_format=torch.channels_last)
        _lib.call("rth_conv_bias_relu", ctypes.byref(nchw_out(shape) if last else shape), hh.data_ptr(), None, n,
                  net._packed_for(packed, li, True).data_ptr(), convs_g[li].bias.data_ptr(), y.data_ptr(),
                  _lib.stream_ptr())
        return y

    def conv_cpu(m, li, h):
        c = m._convs()[li]
        return torch.relu(F.conv2d(h, c.weight, c.bias, stride=c.stride))

    def scale_conv(li, h64):
        c = cpu64._convs()[li]
        return F.conv2d(h64.abs(), c.weight.abs(), stride=c.stride)

    with torch.no_grad():
        w1, b1, w2, b2 = net._merged_head_weights()
        w1c, b1c = w1.detach().cpu(), b1.detach().cpu()

        def heads_cpu(m, h1):
            a2, v2 = m.fc_adv[2], m.fc_value[2]
            H = a2.weight.shape[1]
            return torch.cat([h1[:, :H] @ a2.weight.t() + a2.bias, h1[:, H:] @ v2.weight.t() + v2.bias], 1)

        def fc1_cpu(m, feat):
            a0, v0 = m.fc_adv[0], m.fc_value[0]
            return torch.cat([torch.relu(feat @ a0.weight.t() + a0.bias), torch.relu(feat @ v0.weight.t() + v0.bias)], 1)

        rows = []

        def report(stage, ours, r32, ex, scale, local_ours=None, local_r32=None):
            ex = ex.double()
            e_o = (ours.double().cpu() - ex).abs()
            e_r = (r32.double() - ex).abs()
            row = {"stage": stage, "max_abs_exact": float(ex.abs().max()),
                   "ours_err": float(e_o.max()), "ref32_err": float(e_r.max()),
                   "ours_rel": float((e_o / scale.clamp_min(1e-30)).max()) if scale is not None else None,
                   "ref32_rel": float((e_r / scale.clamp_min(1e-30)).max()) if scale is not None else None}
            if local_ours is not None:
                row["ours_local_err"] = float((local_ours.double().cpu() - ex).abs().max())
                row["ref32_local_err"] = float((local_r32.double() - ex).abs().max())
            rows.append(row)
            print(json.dumps(row), flush=True)

        # ---- torso: propagated and local, stage by stage
        h_g, h_32, h_64 = x8.to(dev), x8.float(), x8.double()
        for li in range(3):
            y_g = conv_gpu(li, h_g)
            y_32 = conv_cpu(cpu32, li, h_32)
            y_64 = conv_cpu(cpu64, li, h_64)
            sc = scale_conv(li, h_64)
            if li == 0:  # the input is exact in every arithmetic: local == propagated
                lo_g, lo_32 = y_g, y_32
            else:
                hx = h_64.float()
                lo_g = conv_gpu(li, hx.to(dev).contiguous(memory_format=torch.channels_last))
                lo_32 = conv_cpu(cpu32, li, hx)
            report(f"conv{li + 1}", y_g.float(), y_32, y_64, sc, lo_g.float(), lo_32)
            h_g, h_32, h_64 = y_g, y_32, y_64
        feat_g, feat_32, feat_64 = h_g.reshape(n, -1), h_32.reshape(n, -1), h_64.reshape(n, -1)
        # ---- FC1 (+ bias + ReLU)
        h1_g = fc1_relu(feat_g, w1, b1)
        h1_32, h1_64 = fc1_cpu(cpu32, feat_32), fc1_cpu(cpu64, feat_64)
        sc1 = feat_64.abs() @ w1c.double().abs().t()
        lo_g = fc1_relu(feat_64.float().to(dev), w1, b1)
        lo_32 = fc1_cpu(cpu32, feat_64.float())
        report("fc1", h1_g, h1_32, h1_64, sc1, lo_g, lo_32)
        # ---- FC2: raw heads [n, A + 1]
        hd_g = net._heads_fc2(h1_g) if w2 is None else torch.addmm(b2, h1_g, w2.t())
        hd_32, hd_64 = heads_cpu(cpu32, h1_32), heads_cpu(cpu64, h1_64)
        H = cpu64.fc_adv[2].weight.shape[1]
        sc2 = torch.cat([h1_64[:, :H].abs() @ cpu64.fc_adv[2].weight.abs().t(),
                         h1_64[:, H:].abs() @ cpu64.fc_value[2].weight.abs().t()], 1)
        lo_g = net._heads_fc2(h1_64.float().to(dev).contiguous()) if w2 is None else \
            torch.addmm(b2, h1_64.float().to(dev), w2.t())
        lo_32 = heads_cpu(cpu32, h1_64.float())
        report("fc2_heads", hd_g, hd_32, hd_64, sc2, lo_g, lo_32)
        # ---- Q(s0, a), target, td (target network = online at init)
        q0_64, tg_64, td_64 = td_of(hd_64[:B], hd_64[B:], hd_64[B:], a_t, r_t.double(), d_t.double(), gamma_n)
        q0_32, tg_32, td_32 = td_of(hd_32[:B], hd_32[B:], hd_32[B:], a_t, r_t, d_t, gamma_n)
        hg = hd_g.detach().cpu()
        q0_g, tg_g, _ = td_of(hg[:B], hg[B:], hg[B:], a_t, r_t, d_t, gamma_n)
        _, td_abs_g, _ = td_huber_forward(hd_g[:B].contiguous(), hd_g[B:].contiguous(), hd_g[B:].contiguous(), a_t, r_t,
                                          d_t, torch.as_tensor(isw), gamma_n, True, False, dueling=True)
        report("q_s0_a", q0_g, q0_32, q0_64, None)
        report("target", tg_g, tg_32, tg_64, None)
        report("abs_td", td_abs_g.cpu(), td_32.abs(), td_64.abs(), None)
        # the fixture's own numbers: ref32 |td| and exact |td| as the reference generator stored them
        print(json.dumps({"fixture": {"ref32_vs_exact": float(np.abs(gd["upd0_abs_td"] - gd["upd0_abs_td64"]).max()),
                                      "ours_vs_fixture_exact": float((td_abs_g.cpu().double() -
                                                                      torch.as_tensor(gd["upd0_abs_td64"])).abs().max()),
                                      "this_exact_vs_fixture_exact": float((td_64.abs() - torch.as_tensor(
                                          gd["upd0_abs_td64"])).abs().max())}}), flush=True)
        if len(sys.argv) > 1:
            with open(sys.argv[1], "w") as f:
                json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
