"""The apex learner's own update at the reference's batch sizes, pinned by the reference.

Golden: tests/golden/dqn_pong_b512.npz (B = 512, A = 6: BASELINE configs[1]'s learner,
test/apex-dqn/config.yaml:2) and dqn_beamrider_b64.npz (B = 64, A = 9: the reference
config's BeamRider, config.yaml:8), each two DQNSolver.update calls of the reference
(reth/reth/algorithm/dqn/dqn_solver.py:104-124) on torch-CPU, with the FULL state_dict
after each (tests/golden/make_golden.py gen_dqn_full).

What runs here is exactly what the bench replays: an ApexDQN (HIP graphs, uint8 batch
slots, the explicit gradient pass of fused_learner.py -- the HIP conv forwards (conv1 bf16x3,
conv2 fp32 MFMA, conv3 x9), FC1's forward on the exact-split rth_fc_x9 with FC2 in its reduce
launch, the fused TD / Huber / FC2 backward, FC1's two backward GEMMs on hipBLASLt, the x9 data
gradients, the fp32 conv2 / conv3 weight gradients, conv1's bf16x3 weight gradient from the
stacks whose reduce launch also finishes the deferred bias / weight gradients and the norm
partials, then Adam) is built with the reference's seed, run until its
graphs are captured, then reset to the initial weights / zero Adam state; the golden batch is
written into a learner batch slot and the captured learner graph is replayed twice.
Tolerances: the first update's |td| within the north-star 1e-5 of the reference's fp32 run
(same weights, same batch), relative to the magnitude of td's operands Q(s0, a) and the TD
target (both ~17 on Pong's unnormalised frames; the fixture holds the float64 target), and in
absolute terms no farther from the exact |td| than 1.5x the reference fp32 run's own distance.  The parameters are compared with the EXACT update (the same
reference code run in float64, stored beside the fp32 run): the reference's own fp32 CPU
update is up to 1.6e-5 away from it on conv1's weight after two updates (Adam's eps = 1.5e-4
turns the fp32 rounding of near-zero gradients into parameter differences), so every tensor
must be at least as close to the exact update as 2x the reference fp32 run's distance, with
the north-star 2e-6 as the floor; the second update's |td| likewise.  Sharper, and free of
Adam's amplification: the first update's gradient (before clipping) against the reference's
fp64 gradient, per tensor within 2x the reference fp32 run's own gradient error + 1e-6 of the
tensor's largest element, and the total norm likewise.  The fixture's seed is
screened (make_golden.py gen_dqn_full): no FC1 ReLU / double-Q argmax decision of the exact
update closer to its threshold than fp32 rounding, where any two fp32 summation orders
(the reference's CPU run included) may decide differently -- one such flip at a relative
margin of 1.3e-8 moved a whole row of FC1's gradient by 2e-3 on the previous seed."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))


@pytest.mark.parametrize("name", ["dqn_pong_b512.npz", "dqn_beamrider_b64.npz"])
def test_apex_learner_graph_vs_reference(golden, dev, name):
    from dqn_batch import apex_batch, frames_sha

    from reth_amd.apex import ApexConfig, ApexDQN

    gd, tag = golden(name), name.split(".")[0]
    B, A, seed = int(gd["B"]), int(gd["A"]), int(gd["seed"])
    s0, s1, a, r, done, isw = apex_batch(seed, B, A)
    assert frames_sha(s0, s1) == str(gd["frames_sha"])
    for x, k in ((a, "a"), (r, "r"), (done, "done"), (isw, "isw")):
        assert np.array_equal(x, gd[k])
    cfg = ApexConfig(n_actors=16, num_actions=A, capacity=max(2048, 2 * B), batch_size=B, sample_start=B, seed=seed,
                     hip_graph=True, update_target_interval=100, send_weights_interval=10 ** 6)
    ax = ApexDQN(cfg, device=dev)
    solver = ax.solver
    names = [str(x) for x in gd["param_names"]]
    sd = solver.q_network.state_dict()
    assert list(sd) == names
    init = {k: v.detach().clone() for k, v in sd.items()}
    sums = np.array([float(v.double().cpu().contiguous().sum()) for v in init.values()])
    np.testing.assert_allclose(sums, gd["init_sum"], rtol=1e-10, atol=1e-9)  # the reference's seeded init
    ax.prefill(cfg.capacity)
    for _ in range(6):
        ax.iteration()
    torch.cuda.synchronize()
    G = ax._graphs
    assert G is not None, "the learner graph was not captured"

    def reset():
        # back to the reference's starting point: initial weights, target = online, fresh Adam
        with torch.no_grad():
            for k, v in solver.q_network.state_dict().items():
                v.copy_(init[k])
            solver.update_target()
            opt = solver.optimizer
            for st in opt.state.values():
                st["exp_avg"].zero_()
                st["exp_avg_sq"].zero_()
            opt._step.zero_()
            opt._ws.zero_()
        p = 0
        cols, idx, w = ax.loader._slots[p]
        cols[0].copy_(torch.as_tensor(s0))
        cols[3].copy_(torch.as_tensor(s1))
        cols[1].copy_(torch.as_tensor(a))
        cols[2].copy_(torch.as_tensor(r))
        cols[4].copy_(torch.as_tensor(done))
        w.copy_(torch.as_tensor(isw))
        torch.cuda.synchronize()
        v = ("full", p)  # the learner computes the target pass itself (as after a target sync)
        stream = torch.cuda.Stream(dev)
        return v, stream

    v, stream = reset()
    report, dump, tds, greport = [], {}, [], []
    pname = {id(p): n for n, p in solver.q_network.named_parameters()}
    stride = int(gd["grad0_row_stride"])
    for k in range(2):
        with torch.cuda.stream(stream):
            ax._learner_replay(v)
        torch.cuda.synchronize()
        td = G["learn_td"][v].double().cpu().numpy()
        td32, td64 = gd[f"upd{k}_abs_td"].astype(np.float64), gd[f"upd{k}_abs_td64"]
        tds.append((k, td, td32, td64))
        if k == 0:  # the gradient this update handed to clip + Adam (rth_clip_adam reads it, const)
            names = [str(x) for x in gd["param_names"]]
            for p, gr in zip(solver._params, G["grads"][v]):
                name = pname[id(p)]
                j = names.index(name)
                ours = gr.double().cpu().numpy()
                if name.startswith("fc_") and name.endswith(".0.weight"):
                    ours = ours[::stride]
                exact = gd[f"grad0_64/{name}"].astype(np.float64)
                assert ours.shape == exact.shape, (name, ours.shape, exact.shape)
                greport.append((name, float(np.abs(ours - exact).max()), float(gd["grad0_ref32_err"][j]),
                                float(gd["grad0_absmax"][j])))
            gnorm = float(solver.optimizer.total_norm.double().cpu())
        for j, (name, t) in enumerate(solver.q_network.state_dict().items()):
            base = init[name].double().cpu()
            exact = base + torch.as_tensor(gd[f"upd{k}_64/{name}"].astype(np.float64))
            ours = t.double().cpu()
            e_ours = float((ours - exact).abs().max())
            e_ref = float(gd[f"upd{k}_ref32_err"][j])
            report.append((k, name, e_ours, e_ref))
            if os.environ.get("RTH_DUMP_LEARNER"):
                dump[f"upd{k}/{name}"] = (ours - base).numpy()
    if os.environ.get("RTH_LEARNER_REPEAT"):  # run-to-run: the same two updates again, bitwise
        first = {k: t.detach().clone() for k, t in solver.q_network.state_dict().items()}
        v, stream = reset()
        for k in range(2):
            with torch.cuda.stream(stream):
                ax._learner_replay(v)
        torch.cuda.synchronize()
        diff = {k: float((t.double() - first[k].double()).abs().max()) for k, t in solver.q_network.state_dict().items()}
        print("repeat: max |run2 - run1| per tensor", {k: f"{d:.1e}" for k, d in diff.items()})
    if dump:
        os.makedirs("gpurun_out", exist_ok=True)
        np.savez_compressed(f"gpurun_out/learner_{tag}.npz", **dump)
    for name, e_ours, e_ref, gmax in greport:
        print(f"update 0 grad {name:20s} |ours - exact| {e_ours:.2e} ({e_ours / gmax:.1e} of max|g|)  "
              f"|ref fp32 - exact| {e_ref:.2e} ({e_ref / gmax:.1e})")
    n64, n32 = float(gd["grad0_norm64"]), float(gd["grad0_norm32"])
    print(f"update 0 grad norm: ours {gnorm:.9e}  exact {n64:.9e}  ref fp32 {n32:.9e}")
    for k, name, e_ours, e_ref in report:
        print(f"update {k} {name:20s} |ours - exact| {e_ours:.2e}  |ref fp32 - exact| {e_ref:.2e}")
    for k, td, td32, td64 in tds:
        ref_td = np.abs(td32 - td64).max()
        print(f"update {k} |td|: |ours - exact| {np.abs(td - td64).max():.2e}  |ref fp32 - exact| {ref_td:.2e}  "
              f"|ours - ref fp32| {np.abs(td - td32).max():.2e} (absolute; north-star bar 1e-5)")
    # the gradient before clipping, update 0 (same weights, same batch: no Adam in between): each
    # tensor within 2x the reference fp32 run's own distance from the exact (fp64) gradient, plus
    # 1e-6 of the tensor's largest element (fp32 summation-order room at the tensor's own scale)
    for name, e_ours, e_ref, gmax in greport:
        assert e_ours <= 2 * e_ref + 1e-6 * gmax, (name, e_ours, e_ref, gmax)
    assert abs(gnorm - n64) <= 2 * abs(n32 - n64) + 1e-6 * n64, (gnorm, n64, n32)
    for k, td, td32, td64 in tds:
        if k == 0:  # same weights, same batch: the north-star 1e-5 against the reference's fp32 run,
            # relative to the operands of td = Q(s0, a) - target (|Q| <= |td| + |target|, ~17 here:
            # the reference's own fp32 run is 1e-5 from the exact |td| in absolute terms) ...
            scale = np.maximum(1.0, td64 + np.abs(gd[f"upd{k}_target64"]))
            rel = np.abs(td - td32) / scale
            assert rel.max() <= 1e-5, (k, rel.max(), int(rel.argmax()))
            # ... and in absolute terms at least nearly as accurate as the reference's own fp32
            # arithmetic: the largest distance from the exact |td| within 1.5x the reference fp32
            # run's (with FC1's 3,136-term single chains on hipBLASLt it was
            # 2.1x, with every FC1 forward on the exact-split GEMM 1.1x)
            e_ours, e_ref = float(np.abs(td - td64).max()), float(np.abs(td32 - td64).max())
            assert e_ours <= 1.5 * e_ref, (k, e_ours, e_ref, e_ours / e_ref)
        ref_td = np.abs(td32 - td64).max()
        assert np.abs(td - td64).max() <= 2 * ref_td + 1e-5, (k, np.abs(td - td64).max(), ref_td)
    for k, name, e_ours, e_ref in report:
        # at least as close to the exact (fp64) update as 2x the reference's own fp32 CPU run,
        # within the north-star 2e-6 floor (+ the fixture's float16 rounding, 2 x 1.5e-7)
        assert e_ours <= 2 * e_ref + 2e-6 + 3e-7, (k, name, e_ours, e_ref)
    ax.close()
