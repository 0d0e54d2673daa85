"""The learner's gradient pass for the dueling Nature-DQN as an explicit kernel sequence.

Reference: reth/reth/algorithm/dqn/dqn_solver.py:68-117 (_calc_td_error, then
loss.backward()) on reth/reth/algorithm/dqn/dqn_model.py:6-56.  Same math as the autograd
path of solver.py (compute_grads with torch.autograd), without the autograd engine's glue:

  forward   Q(s0) and Q(s1) of the online network as ONE pass over 2B stacks (the batch
            slot keeps s1 right behind s0, replay.HbmReplay.new_batch), each conv one
            rth_conv_bias_relu launch (the last one writes NCHW: FC1 reads the reference's
            (C, H, W) flatten order), FC1 one hipBLASLt GEMM with the bias+ReLU epilogue on
            the tied [2H, F] parameter storage (model._tie_heads), FC2 one rth_heads_fc2
            launch on the branch parameters in place;
  TD        rth_td_huber on the raw heads -> |td|, loss, d(loss)/d(heads of s0), fused with
  backward  FC2 + threshold + both bias sums (rth_td_heads_backward_branches: FC2's
            gradients written in branch form; also the Trainer's mean |td|), FC1 as two
            GEMMs (its branch gradients are row slices of the merged ones), conv3 as
            rth_relu_bias_grad_nchw + MIOpen's data and weight gradients, conv2 as
            rth_relu_bias_grad + rth_conv_dgrad + MIOpen's weight gradient, conv1 as
            rth_conv_relu_wgrad straight from the uint8 stacks (f32 input:
            rth_relu_bias_grad + MIOpen's weight gradient).  No merged copy of the heads is
            built or split per update.

Only the first B rows of the 2B forward are differentiated: they are contiguous views
(NHWC, batch-major), so the backward reads them in place.
"""
import torch

from . import _lib
from ._lib import call, ctypes, ptr, stream_ptr
from . import model
from .model import fc1_relu, nchw_out
from .replay import FrameStacks


TD_HB_MAX = 16384  # rth_td_heads_backward keeps B * (A + 1) TD gradient rows in LDS
# Module constants (tests patch them to run the alternative kernels; no environment switches):
# HIP_DGRAD -- the layers whose data gradient runs on rth_conv_dgrad (the exact-split bf16 MFMA,
# no zero fill) instead of MIOpen: conv2's (4 stride-parity classes in one launch) and conv3's
# (0.570-0.574 vs 0.575-0.580 ms/step with MIOpen's, r04).
HIP_DGRAD = {1, 2}
# HIP_WGRAD -- the conv2 / conv3 weight gradients: "f32" = rth_conv_wgrad_f32 (the default since
# r06: fp32 MFMA, register-only, fixed summation order -- run-to-run deterministic, no zero fill;
# with uint8 input its split partials are reduced by conv1's reduce launch; step equal to
# MIOpen's, 0.516-0.518 vs 0.515-0.516 ms, whose solvers differ in the last bits run to run and
# whose find picks differ box to box), "x9" = rth_conv_wgrad_x9 (bf16 MFMA, exact 3 x 3-term
# split, deterministic), None = MIOpen's solver + zero fill
HIP_WGRAD = "f32"
# DGRAD_PREPACK -- the data gradients' flipped kernels packed in the forward's pack launch
# (rth_conv_pack_many with CONV_PACK_DGRAD jobs) instead of one pack launch per data gradient
DGRAD_PREPACK = True
# DGRAD_MASK -- conv3's data gradient applies conv2's ReLU mask and writes conv2's bias-gradient
# slabs in its own epilogue (rth_conv_dgrad_relu_prepacked): one launch fewer per update
DGRAD_MASK = True
# NORM_IN_BACKWARD -- one rank, ClipAdam: clip_grad_norm_'s partials written by conv1's
# weight-gradient reduce launch (extra workgroups over the gradients final before it, and the
# squares of what it finishes itself), so the optimizer step is rth_adam_prenormed alone (r06)
NORM_IN_BACKWARD = True


def _net_workspace(net, kind, shape, device):
    """a backward kernel's workspace, owned by the network: two learners in one process may
    run (or replay) their backward passes on different streams, so no workspace is shared
    between them -- rth_conv_dgrad_ws's packed flipped kernel, rth_conv_wgrad_{f32,x9}'s
    split partials, rth_conv_relu_wgrad's conv1 partials"""
    cache = net.__dict__.setdefault("_bwd_ws", {})
    key = (device, kind, shape.input, shape.cin, shape.hin, shape.cout)
    ws = cache.get(key)
    if ws is None:
        fn = {"dgrad": "rth_conv_dgrad_workspace", "conv1": "rth_conv_wgrad_workspace"}.get(
            kind, f"rth_conv_wgrad_{kind}_workspace")
        size = getattr(_lib.lib(), fn)(ctypes.byref(shape))
        ws = cache[key] = torch.empty(max(size, 16) // 4, dtype=torch.float32, device=device)
    return ws


def eligible(net, s0, s1):
    """the explicit pass covers the channels-last dueling net whose three convs all run in
    rth_conv_bias_relu, on uint8 stacks or f32 channels-last observations"""
    if not (getattr(net, "dueling", False) and getattr(net, "hwc_features", False) and getattr(net, "hip_conv", False)):
        return False
    frames = isinstance(s0, FrameStacks), isinstance(s1, FrameStacks)
    if any(frames):  # frames in place: conv1 reads the frame store by the batch's frame ids
        return all(frames) and s0.shape == s1.shape and all(
            sh is not None for _, sh in net._torso_shapes(tuple(s0.shape[1:]), True))
    if not (torch.is_tensor(s0) and torch.is_tensor(s1) and s0.is_cuda and s1.is_cuda and s0.dtype == s1.dtype):
        return False
    if s0.dtype not in (torch.uint8, torch.float32) or s0.shape != s1.shape or s0.dim() != 4:
        return False
    shapes = net._torso_shapes(tuple(s0.shape[1:]), s0.dtype == torch.uint8)
    return all(sh is not None for _, sh in shapes)


def _pair(s0, s1):
    """[s0; s1] as one [2B, ...] tensor: a view when s1 sits right behind s0 in memory (the
    apex batch slots), else a copy"""
    u8 = s0.dtype == torch.uint8
    fmt = torch.contiguous_format if u8 else torch.channels_last
    if s0.is_contiguous(memory_format=fmt) and s1.is_contiguous(memory_format=fmt) and s1.stride() == s0.stride() \
            and s1.untyped_storage().data_ptr() == s0.untyped_storage().data_ptr() \
            and s1.data_ptr() == s0.data_ptr() + s0.numel() * s0.element_size():
        return torch.as_strided(s0, (2 * s0.shape[0], *s0.shape[1:]), s0.stride())
    return torch.cat([s0, s1]).contiguous(memory_format=fmt)


def _nhwc(t):
    return t if t.is_contiguous(memory_format=torch.channels_last) else t.contiguous(memory_format=torch.channels_last)


def dueling_grads(solver, s0, a, r, s1, done, isw, q1t=None, td_acc=None, mid=None, probe=None, prenorm=False):
    """forward + TD + backward of one learner batch; sets .grad of every online parameter
    and returns (loss [], |td| [B]).  q1t: the target network's heads on s1 if precomputed
    (DQNSolver.target_heads).  td_acc (nullable f32 device scalar): += mean |td|.

    mid (optional callable) is handed each gradient bucket as soon as it is final: first the
    heads' [gw1, gb1, gwa2, gwv2, gba2, gbv2] (before the conv backward; the FC1 branch
    gradients are row slices of gw1 / gb1), then the conv weights' and biases'.  The data-parallel
    capture ends a graph there, so the all-reduce of the first bucket overlaps the conv
    backward; whatever mid's caller does to a bucket in place is what the parameters get.

    probe (optional callable) is handed the forward's conv2 and conv3 launches as
    probe([("conv2", launch2), ("conv3", launch3)]), then the fused TD/heads backward as
    probe([("td_heads_backward", launch)]), and issues them itself (the bench times them live:
    the capture cuts the learner graph at each probe, and every replay of that probe graph
    launches them eagerly between HIP events on the learner stream; their buffers live in the
    graph's pool at fixed addresses)."""
    from .solver import td_huber_forward

    net = solver.q_network
    B = s0.shape[0]
    u8 = s0.dtype == torch.uint8
    frames = isinstance(s0, FrameStacks)  # conv1 (forward, weight gradient) reads the frame store
    pair = bool(solver.double_q)
    if frames:
        x = FrameStacks.pair(s0, s1) if pair else s0
    else:
        x = _pair(s0, s1) if pair else (s0 if u8 else _nhwc(s0))
    n = x.shape[0]
    convs = net._convs()
    shapes = [sh for _, sh in net._torso_shapes(tuple(s0.shape[1:]), u8)]
    with torch.no_grad():
        w1, b1, w2, b2 = net._merged_head_weights()  # FC1: the tied parameter storage
        hp = net._head_params()
        fc2p = (_lib.c_vp * 4)(*[p.data_ptr() for p in hp[4:]])  # FC2 read in place
        # the packed data-gradient kernels of this iteration's weights (the backward reads the
        # same weights as the forward: the optimizer steps after both), packed in the forward's
        # pack launch
        dgp, extra = {}, []
        if DGRAD_PREPACK:
            for li in HIP_DGRAD:
                sh = shapes[li] if li < len(shapes) else None
                if sh is None or _lib.lib().rth_conv_dgrad_workspace(ctypes.byref(sh)) <= 0:
                    continue
                dgp[li] = _net_workspace(net, "dgrad", sh, x.device)
                flagged = _lib.ConvShape(sh.input | _lib.CONV_PACK_DGRAD, sh.cin, sh.hin, sh.win, sh.cout, sh.kh, sh.kw,
                                         sh.stride)
                extra.append((flagged, _nhwc(convs[li].weight.detach()).data_ptr(), dgp[li].data_ptr()))
        packed = net.pack_convs(u8=u8, extra=extra)
        st = stream_ptr()
        ys, h = [], x
        probed = []  # [(tag, launch)] of conv2 / conv3, handed to probe together
        for li, (conv, shape) in enumerate(zip(convs, shapes)):
            last = li == len(convs) - 1  # writes NCHW: FC1 reads the (C, H, W) flatten order
            ho = (shape.hin - shape.kh) // shape.stride + 1
            wo = (shape.win - shape.kw) // shape.stride + 1
            y = torch.empty((n, shape.cout, ho, wo), dtype=torch.float32, device=x.device,
                            memory_format=torch.contiguous_format if last else torch.channels_last)
            def launch(shape=nchw_out(shape) if last else shape, h=h, pk=net._packed_for(packed, li, u8),
                       b=conv.bias, y=y):
                if isinstance(h, FrameStacks):
                    call("rth_conv1_frames_bias_relu", ctypes.byref(shape), ptr(h.store), ptr(h.ids), n, ptr(pk),
                         ptr(b), ptr(y), stream_ptr())
                else:
                    call("rth_conv_bias_relu", ctypes.byref(shape), ptr(h), None, n, ptr(pk), ptr(b), ptr(y),
                         stream_ptr())

            if probe is not None and li in (1, 2):
                probed.append((f"conv{li + 1}", launch))
                if li == min(2, len(convs) - 1):  # one cut for both: the prober issues them, in order
                    probe(probed)
            else:
                launch()
            ys.append(y)
            h = y
        feat = h.view(n, -1)  # the (C, H, W) flatten of the NCHW output: a view
        h1 = heads = None
        if w2 is None and model.FC1_HEADS:  # FC1's reduce + FC2 in one launch, h1 kept for the backward
            h1 = torch.empty((feat.shape[0], w1.shape[0]), dtype=torch.float32, device=feat.device)
            heads = net._fc1_heads(feat, w1, b1, h1_out=h1)
        if heads is None:
            h1 = fc1_relu(feat, w1, b1, owner=net)
            heads = net._heads_fc2(h1) if w2 is None else torch.addmm(b2, h1, w2.t())
        if q1t is None:
            q1t = solver.target_heads(s1)
        q0 = heads[:B]
        q1o = heads[B:] if pair else None
        H2, A1 = w1.shape[0], hp[4].shape[0] + 1
        Hh = H2 // 2
        gh1 = torch.empty((B, H2), dtype=torch.float32, device=x.device)
        gb1 = torch.empty_like(b1)
        g2 = [torch.empty_like(p) for p in hp[4:]]  # the second layer's gradients, branch form
        g2p = (_lib.c_vp * 4)(*[t.data_ptr() for t in g2])
        if B * A1 <= TD_HB_MAX:
            # TD/Huber + FC2 + threshold + bias sums in one launch
            dev = x.device
            a = a.to(device=dev, dtype=torch.int64).contiguous().view(-1)
            r = r.to(device=dev, dtype=torch.float32).contiguous().view(-1)
            done = done.to(device=dev, dtype=torch.float32).contiguous().view(-1)
            if isw is not None:
                isw = isw.to(device=dev, dtype=torch.float64).contiguous().view(-1)
            q1t = q1t.contiguous()
            if q1t.shape != q0.shape or a.numel() != B or r.numel() != B or done.numel() != B or \
                    (isw is not None and isw.numel() != B):
                raise ValueError("batch columns / target heads disagree with the batch")
            td_abs = torch.empty(B, dtype=torch.float32, device=dev)
            loss = torch.empty(1, dtype=torch.float32, device=dev)
            def td_launch(q1t=q1t, a=a, r=r, done=done, isw=isw):
                call("rth_td_heads_backward_branches", ptr(q0), ptr(q1o), ptr(q1t), ptr(a), ptr(r), ptr(done), ptr(isw),
                     B, A1 - 1, float(solver.gamma_n), int(bool(solver.double_q)), ptr(h1), h1.stride(0), fc2p, Hh,
                     ptr(td_abs), ptr(loss), ptr(gh1), g2p, ptr(gb1), ptr(td_acc), stream_ptr())

            if probe is not None:
                probe([("td_heads_backward", td_launch)])
            else:
                td_launch()
        else:
            loss, td_abs, dq = td_huber_forward(q0, q1o, q1t, a, r, done, isw, solver.gamma_n, solver.double_q,
                                                want_dq=True, dueling=True)
            # FC2 + threshold + bias sums
            call("rth_heads_backward_branches", ptr(dq), ptr(h1), h1.stride(0), fc2p, Hh, B, A1 - 1, ptr(gh1), g2p,
                 ptr(gb1), ptr(td_abs), ptr(td_acc), st)
        # FC1
        gfeat = torch.mm(gh1, w1)
        gw1 = torch.mm(gh1.t(), feat[:B])
        if mid is not None:
            mid([gw1, gb1, *g2])
        g = gfeat.view(ys[-1][:B].shape)  # NCHW, like the last conv's output
        grads = {}
        deferred = []  # bias gradients whose slabs wait for conv1's reduce launch
        wdeferred = []  # conv2 / conv3 weight gradients whose partials wait for it (HIP_WGRAD "f32")
        if getattr(net, "_ws", None) is None or net._ws[0].device != x.device:
            net._ws = [torch.zeros(_lib.lib().rth_relu_bias_grad_workspace(m.out_channels), dtype=torch.uint8,
                                   device=x.device) for m in convs]
        fused_below = None  # (masked gradient, db) of the layer below, from the fused data gradient
        for li in range(len(convs) - 1, -1, -1):
            conv, y = convs[li], ys[li][:B]
            if li == 0 and u8:  # ReLU mask + weight/bias gradients from the stacks, and the
                # deferred conv3 / conv2 bias gradients in the same reduce launch
                gw = torch.empty(conv.weight.shape, dtype=torch.float32, device=x.device,
                                 memory_format=torch.channels_last)
                db = torch.empty(conv.out_channels, dtype=torch.float32, device=x.device)
                assert len(deferred) <= 4, "rth_conv_relu_wgrad_ex finishes at most 4 deferred bias gradients"
                jobs = (_lib.BiasDeferred * max(len(deferred), 1))(*deferred)
                wjobs = (_lib.WgradDeferred * max(len(wdeferred), 1))(*wdeferred)
                ws1 = _net_workspace(net, "conv1", shapes[0], x.device)
                opt = solver.optimizer
                if prenorm and NORM_IN_BACKWARD and mid is None and solver.grad_hook is None and hasattr(opt, "prenorm"):
                    # every gradient but conv1's weight and bias and the deferred biases (this
                    # launch finishes those) is final here: the heads' and conv2 / conv3's weights
                    done = {d.db for d in deferred} | {d.gw for d in wdeferred}
                    sq = [gr for gr in [gw1[:Hh], gw1[Hh:], gb1[:Hh], gb1[Hh:], *g2]]
                    sq += [gr for c in convs[1:] for gr in (grads[c.weight], grads[c.bias])
                           if gr.data_ptr() not in done]
                    arr, n_sq = opt.norm_tensors(sq)
                    nparts = ctypes.c_int32(0)
                    call("rth_conv1_relu_wgrad_norm", ctypes.byref(shapes[0]), ptr(x.store) if frames else ptr(x), None,
                         ptr(x.ids) if frames else None, B, ptr(_nhwc(g)), ptr(y), ptr(gw), ptr(db), ptr(ws1), jobs,
                         len(deferred), wjobs, len(wdeferred), arr, n_sq, *opt.prenorm_scalars(),
                         ctypes.byref(nparts), st)
                    opt.prenorm(nparts.value)
                elif frames:
                    call("rth_conv1_frames_relu_wgrad_ex", ctypes.byref(shapes[0]), ptr(x.store), ptr(x.ids), B,
                         ptr(_nhwc(g)), ptr(y), ptr(gw), ptr(db), ptr(ws1), jobs, len(deferred), wjobs,
                         len(wdeferred), st)
                else:
                    call("rth_conv_relu_wgrad_ex", ctypes.byref(shapes[0]), ptr(x), None, B, ptr(_nhwc(g)), ptr(y),
                         ptr(gw), ptr(db), ptr(ws1), jobs, len(deferred), wjobs, len(wdeferred), st)
                grads[conv.weight], grads[conv.bias] = gw, db
                deferred, wdeferred = [], []  # consumed
                break
            nb, c, hh, ww = y.shape
            defer = u8  # finished by conv1's rth_conv_relu_wgrad_ex
            if fused_below is not None:  # masked and its bias slabs written by the data gradient above
                gy, db = fused_below
                fused_below = None
            else:
                gy = torch.empty((nb, c, hh, ww), dtype=torch.float32, device=x.device,
                                 memory_format=torch.channels_last)
                db = torch.empty(c, dtype=torch.float32, device=x.device)
                if li == len(convs) - 1:  # NCHW output: mask + bias partials, gy written channels-last
                    call("rth_relu_bias_grad_nchw", ptr(g), ptr(y), ptr(gy), None if defer else ptr(db),
                         ptr(net._ws[li]), nb, c, hh * ww, st)
                else:
                    g = _nhwc(g)
                    call("rth_relu_bias_grad", ptr(g), ptr(y), ptr(gy), None if defer else ptr(db), ptr(net._ws[li]),
                         nb * hh * ww, c, st)
                if defer:
                    deferred.append(_lib.BiasDeferred(net._ws[li].data_ptr(), db.data_ptr(), nb * hh * ww, c, 0))
            xin = ys[li - 1][:B] if li > 0 else x[:B]
            w = _nhwc(conv.weight.detach())
            hip_dgrad = li in HIP_DGRAD and _lib.lib().rth_conv_dgrad_supported(ctypes.byref(shapes[li]))
            hip_wgrad = bool(HIP_WGRAD) and getattr(_lib.lib(), f"rth_conv_wgrad_{HIP_WGRAD}_supported")(
                ctypes.byref(shapes[li]))
            need = [li > 0 and not hip_dgrad, not hip_wgrad, False]
            gx = gw = None
            if need[0] or need[1]:
                gx, gw, _ = torch.ops.aten.convolution_backward(gy, xin, w, None, list(conv.stride), [0, 0], [1, 1],
                                                                False, [0, 0], 1, need)
            if hip_wgrad:  # weight gradient in rth_conv_wgrad_{f32,x9} (deterministic, no zero fill)
                gw = torch.empty(conv.weight.shape, dtype=torch.float32, device=x.device,
                                 memory_format=torch.channels_last)
                ws = _net_workspace(net, HIP_WGRAD, shapes[li], x.device)
                if HIP_WGRAD == "f32" and defer:  # partials now, the reduce in conv1's reduce launch
                    job = _lib.WgradDeferred()
                    call("rth_conv_wgrad_f32_partials", ctypes.byref(shapes[li]), ptr(xin), B, ptr(gy), ptr(gw), ptr(ws),
                         ctypes.byref(job), st)
                    wdeferred.append(job)
                else:
                    call(f"rth_conv_wgrad_{HIP_WGRAD}", ctypes.byref(shapes[li]), ptr(xin), B, ptr(gy), ptr(gw), ptr(ws),
                         st)
            if hip_dgrad:  # data gradient in rth_conv_dgrad (no zero fill)
                gx = torch.empty(xin.shape, dtype=torch.float32, device=x.device, memory_format=torch.channels_last)
                if li in dgp and li > 0 and defer and DGRAD_MASK and \
                        _lib.lib().rth_conv_dgrad_relu_supported(ctypes.byref(shapes[li])):
                    # + the layer below's ReLU mask and bias slabs (its rth_relu_bias_grad launch)
                    slabs = ctypes.c_int64(0)
                    call("rth_conv_dgrad_relu_prepacked", ctypes.byref(shapes[li]), ptr(gy), B, ptr(dgp[li]), ptr(xin),
                         ptr(gx), ptr(net._ws[li - 1]), ctypes.byref(slabs), st)
                    cb = convs[li - 1].out_channels
                    db_below = torch.empty(cb, dtype=torch.float32, device=x.device)
                    deferred.append(_lib.BiasDeferred(net._ws[li - 1].data_ptr(), db_below.data_ptr(),
                                                      xin.shape[0] * xin.shape[2] * xin.shape[3], cb, slabs.value))
                    fused_below = (gx, db_below)
                elif li in dgp:  # packed in the forward's pack launch
                    call("rth_conv_dgrad_prepacked", ctypes.byref(shapes[li]), ptr(gy), B, ptr(dgp[li]), ptr(gx), st)
                else:
                    call("rth_conv_dgrad_ws", ctypes.byref(shapes[li]), ptr(gy), B, ptr(w), ptr(gx),
                         ptr(_net_workspace(net, "dgrad", shapes[li], x.device)), st)
            grads[conv.weight], grads[conv.bias] = gw, db
            g = gx
        # every deferred bias gradient was finished by conv1's launch (else its db would be
        # uninitialised memory handed to the optimizer)
        assert not deferred and not wdeferred, "deferred bias / weight gradients left unfinished"
        if mid is not None:
            mid([t for c in convs for t in (grads[c.weight], grads[c.bias])])
        # the eight branch parameters' gradients: FC1's are row slices of the merged ones (the
        # parameters are row slices of one storage, model._tie_heads), FC2's were written in
        # branch form by the heads' backward
        for p, gr in zip(hp, [gw1[:Hh], gw1[Hh:], gb1[:Hh], gb1[Hh:], *g2]):
            grads[p] = gr
    for p in net.parameters():
        p.grad = grads[p]
    return loss.view(()), td_abs
