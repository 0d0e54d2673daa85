"""Q-networks (PyTorch-ROCm; MIOpen / hipBLASLt run the conv and linear GEMMs in fp32).

Parameter names, shapes and the order in which modules are constructed match
reth/reth/algorithm/dqn/dqn_model.py:6-71, so
  * state_dicts (and torch.save weight streams, dqn_solver.py:133-143) are interchangeable
    with the reference's, and
  * under the same torch.manual_seed the default initialisation is identical.
"""

import torch
from torch import nn


def conv_out(size, k, s):
    return (size - k) // s + 1


def nchw_out(shape):
    """a copy of an rth_conv_shape with RTH_CONV_OUT_NCHW set (the conv writes NCHW)"""
    from ._lib import CONV_OUT_NCHW, ConvShape

    return ConvShape(shape.input | CONV_OUT_NCHW, shape.cin, shape.hin, shape.win, shape.cout, shape.kh, shape.kw,
                     shape.stride)


class DQNNetwork(nn.Module):
    """Nature-DQN torso + dueling heads (dqn_model.py:6-56): obs (C, H, W) -> Q[A]."""

    def __init__(self, obs_shape, num_actions, dueling=True, hidden_unit=256):
        super().__init__()
        c, h, w = obs_shape
        self.input_shape, self.num_actions, self.dueling = tuple(obs_shape), num_actions, dueling
        self.features = nn.Sequential(
            nn.Conv2d(c, 32, kernel_size=8, stride=4), nn.ReLU(),
            nn.Conv2d(32, 64, kernel_size=4, stride=2), nn.ReLU(),
            nn.Conv2d(64, 64, kernel_size=3, stride=1), nn.ReLU())
        fh = conv_out(conv_out(conv_out(h, 8, 4), 4, 2), 3, 1)
        fw = conv_out(conv_out(conv_out(w, 8, 4), 4, 2), 3, 1)
        nfeat = 64 * fh * fw
        self._feat_chw = (64, fh, fw)
        # forward_heads on channels-last input: HIP conv epilogues and NHWC feature order
        self.hwc_features = False
        self.hip_conv = True  # rth_conv_bias_relu for the built torso geometries (else MIOpen)
        if dueling:
            self.fc_adv = nn.Sequential(nn.Linear(nfeat, hidden_unit), nn.ReLU(), nn.Linear(hidden_unit, num_actions))
            self.fc_value = nn.Sequential(nn.Linear(nfeat, hidden_unit), nn.ReLU(), nn.Linear(hidden_unit, 1))
            self._tie_heads()
        else:
            self.fc = nn.Sequential(nn.Linear(nfeat, 512), nn.ReLU(), nn.Linear(512, num_actions))

    def _tie_heads(self):
        """FC1 of the two dueling branches as the row slices [0, H) / [H, 2H) of ONE [2H, F]
        weight storage (and their biases of one [2H]): the merged FC1 that the fast path
        multiplies by is the parameters themselves, read and updated in place (no merge or
        split launch per update).  Parameter objects, names, shapes and values are unchanged
        (state_dict, optimizers and torch.save streams see the reference's eight tensors);
        re-tied after every device / dtype move (_apply)."""
        a0, v0 = self.fc_adv[0], self.fc_value[0]
        H = a0.weight.shape[0]
        w = torch.cat([a0.weight.detach(), v0.weight.detach()])
        b = torch.cat([a0.bias.detach(), v0.bias.detach()])
        a0.weight.data, v0.weight.data = w[:H], w[H:]
        a0.bias.data, v0.bias.data = b[:H], b[H:]
        self._w1s, self._b1s = w, b

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        if self.dueling:
            self._tie_heads()
        return out

    def _tie_check(self):
        """re-tie FC1 when something replaced the branch parameters' storage (copy.deepcopy,
        load_state_dict(assign=True), vector_to_parameters): the fast path multiplies by
        _w1s / _b1s, which must be the storage the two parameters are views of"""
        if not self.dueling:
            return
        a0, v0 = self.fc_adv[0], self.fc_value[0]
        w, b = self.__dict__.get("_w1s"), self.__dict__.get("_b1s")
        H = a0.weight.shape[0]
        ok = (w is not None and b is not None and a0.weight.data_ptr() == w.data_ptr()
              and v0.weight.data_ptr() == w[H:].data_ptr() and a0.bias.data_ptr() == b.data_ptr()
              and v0.bias.data_ptr() == b[H:].data_ptr() and w.device == a0.weight.device)
        if not ok:
            self._tie_heads()

    def __deepcopy__(self, memo):
        """deepcopy clones every Parameter into its own storage: re-tie FC1 in the copy (the
        cached head / packed weights are per-object state and are not carried over)"""
        import copy

        new = self.__class__.__new__(self.__class__)
        memo[id(self)] = new
        skip = ("_w1s", "_b1s", "_frozen", "_frozen_packed", "_ws", "_shape_cache", "_fc_ws", "_bwd_ws")
        for k, v in self.__dict__.items():
            if k not in skip:
                new.__dict__[k] = copy.deepcopy(v, memo)
        if new.dueling:
            new._tie_heads()
        return new

    def forward(self, x):
        x = self.features(x).flatten(1)
        if not self.dueling:
            return self.fc(x)
        adv = self.fc_adv(x)
        value = self.fc_value(x)
        return value + adv - adv.mean(dim=1, keepdim=True)  # (value + adv) - mean, :192-193

    # ---------------------------------------------------------------- fused heads path
    # The same function with the two dueling branches merged: FC1 of both branches is one
    # 3136 -> 512 GEMM with the bias and ReLU fused into hipBLASLt's epilogue (its weight is
    # the tied [2H, F] storage, _tie_heads; the features in the reference's (C, H, W) flatten
    # order: the last HIP conv writes NCHW), and the two output layers are one 512 -> A+1
    # launch reading the branch parameters in place (rth_heads_fc2; block-diagonal).  It returns the raw heads [B, A+1] = (advantages, value); the HIP
    # consumers (rth_td_huber, rth_eps_greedy in dueling mode) form Q = (V + A) - mean(A)
    # themselves.  Under autograd the merged weights are a differentiable function of the
    # eight parameters (a copy, block-diagonal FC2 as one GEMM); otherwise nothing is built.
    def _head_params(self):
        a0, v0, a2, v2 = self.fc_adv[0], self.fc_value[0], self.fc_adv[2], self.fc_value[2]
        return [a0.weight, v0.weight, a0.bias, v0.bias, a2.weight, v2.weight, a2.bias, v2.bias]

    def _merged_head_weights(self):
        """(w1, b1, w2, b2) of the merged heads.  Under autograd (a parameter requires grad) a
        differentiable copy built from the eight parameters; otherwise w1 / b1 are the tied
        storage itself and, on the GPU, w2 / b2 are None: the second layer is read from the
        branch parameters in place (rth_heads_fc2 / rth_td_heads_backward_branches)."""
        ps = self._head_params()
        a0, v0, a2, v2 = self.fc_adv[0], self.fc_value[0], self.fc_adv[2], self.fc_value[2]
        A, H = a2.weight.shape
        if torch.is_grad_enabled() and any(p.requires_grad for p in ps):
            if ps[0].is_cuda:  # one HIP launch (and one for the gradients), qnet.hip
                return _MergeHeads.apply((H, ps[0].shape[1], A, 0, 1), *ps)
            w1, b1 = torch.cat([a0.weight, v0.weight]), torch.cat([a0.bias, v0.bias])
        else:
            self._tie_check()
            w1, b1 = self._w1s, self._b1s
            if ps[0].is_cuda and self._fc2_inplace():
                return w1, b1, None, None
        w2 = torch.cat([torch.cat([a2.weight, a2.weight.new_zeros(A, H)], 1),
                        torch.cat([v2.weight.new_zeros(1, H), v2.weight], 1)])
        b2 = torch.cat([a2.bias, v2.bias])
        return w1, b1, w2, b2

    def _fc2_inplace(self):
        """rth_heads_fc2's built shapes: up to 32 actions (every Atari action set: Pong 6,
        Breakout 4, BeamRider 9, the full 18), H a multiple of 64 up to 512"""
        A, H = self.fc_adv[2].weight.shape
        return A <= 32 and H % 64 == 0 and H <= 512

    def _heads_fc2(self, h):
        """the second layer on h = relu(FC1) [n, 2H] from the branch parameters in place
        (rth_heads_fc2): raw heads [n, A+1]"""
        from ._lib import c_vp, call, ptr, stream_ptr

        ps = self._head_params()[4:]
        A, H = ps[0].shape
        out = torch.empty((h.shape[0], A + 1), dtype=torch.float32, device=h.device)
        arr = (c_vp * 4)(*[p.data_ptr() for p in ps])
        call("rth_heads_fc2", ptr(h), h.stride(0), h.shape[0], H, A, arr, ptr(out), stream_ptr())
        return out

    def _fc1_heads(self, h, w1, b1, h1_out=None):
        """FC1 -> FC2 of both branches in rth_fc1_heads (the x9 GEMM, then its split-K reduce +
        bias + ReLU and the second layer in one launch, r06; bit-identical to rth_fc_x9 +
        rth_heads_fc2) where built for the shape, else None.  h1_out (optional [n, 2H]) receives
        relu(FC1) (the learner's backward reads it)"""
        from ._lib import c_vp, call, lib, ptr, stream_ptr

        if not (h.is_cuda and h.dim() == 2 and h.stride(1) == 1 and w1.is_contiguous() and self._fc2_inplace()):
            return None
        M, K = h.shape
        N = w1.shape[0]
        ps = self._head_params()[4:]
        A, H = ps[0].shape
        if N != 2 * H or not lib().rth_fc1_heads_supported(M, N, K, A):
            return None
        out = torch.empty((M, A + 1), dtype=torch.float32, device=h.device)
        arr = (c_vp * 4)(*[p.data_ptr() for p in ps])
        ws = _fc_workspace("rth_fc_x9", h.device, w1, M, N, K, self)
        call("rth_fc1_heads", ptr(h), h.stride(0), M, ptr(w1), N, K, ptr(b1), A, arr, ptr(out),
             ptr(h1_out) if h1_out is not None else None, ptr(ws), stream_ptr())
        return out

    @torch.no_grad()
    def freeze_heads(self):
        """(re)build the cached head weights and packed conv weights IN PLACE (stable storage
        for graph replay): for copies whose parameters change only at refresh points (target
        sync, actor weight reload).  FC1 is the tied parameter storage and, where
        rth_heads_fc2 is built, the second layer is read from its parameters in place; the
        merged second layer of other shapes is rebuilt into the tensors the first freeze
        allocated, whose addresses captured graphs hold."""
        self._tie_check()
        merged = list(self._merged_head_weights())
        old = getattr(self, "_frozen", None)
        if old is not None:
            for k in (2, 3):
                if old[k] is not None and merged[k] is not None and old[k].shape == merged[k].shape:
                    old[k].copy_(merged[k])
                    merged[k] = old[k]
        self._frozen = merged
        if self.hwc_features and self._frozen[0].is_cuda:
            self._frozen_packed = self.pack_convs(out=getattr(self, "_frozen_packed", None))

    def forward_heads(self, x, merged=None, rows=None, packed=None, n_dev=None, n_fixed=None, cache=None):
        """raw dueling heads [n, A+1].  x: float32 observations (channels-last with
        hwc_features), or -- on the HIP torso -- uint8 frame stacks [m, C, H, W], read as
        stacks `rows` (an int64 device index, n = rows.numel()) or all m of them.  merged /
        packed: the head weights / packed conv weights of this weight version (pack_convs),
        default the frozen ones, else built now.  n_dev (int64 device scalar, inference only):
        only the first *n_dev of the n samples are computed by the torso (rows past it hold
        whatever the FC layers make of unwritten activations).  n_fixed (with n_dev, the
        in-place second layer): the first n_fixed rows are always live -- FC1 runs as a
        library GEMM over those only, the counted rows behind them through
        rth_linear_relu_rows_upto, the second layer over the counted rows only; rows past
        *n_dev of the result are undefined.  cache = (heads cache [stacks, A+1], rows int64
        [n]) also receives the counted rows' heads at their stack rows (same launch)."""
        if not self.dueling:
            raise ValueError("forward_heads needs the dueling network")
        frozen = getattr(self, "_frozen", None) is not None
        if merged is None:
            merged = self._frozen if frozen else self._merged_head_weights()
        w1, b1, w2, b2 = merged
        if self.hwc_features:
            if packed is None and frozen:
                packed = getattr(self, "_frozen_packed", None)
            h = self._features_nhwc(x, rows, packed, n_dev)
        else:
            if x.dtype == torch.uint8 or rows is not None or n_dev is not None:
                raise ValueError("uint8 / row-indexed / counted observations need the HIP torso (hwc_features)")
            h = self.features(x)
        h = h.reshape(h.shape[0], -1)  # (C, H, W) flatten: a view of the last HIP conv's NCHW output
        if n_dev is not None and w2 is None and (n_fixed is not None or cache is not None):
            return self._heads_counted(h, w1, b1, n_dev, n_fixed, cache)
        if cache is not None or n_fixed is not None:
            raise ValueError("forward_heads(cache= / n_fixed=) needs n_dev and the in-place second layer")
        if w2 is None and FC1_HEADS and not (torch.is_grad_enabled() and (h.requires_grad or w1.requires_grad)):
            out = self._fc1_heads(h, w1, b1)  # inference: FC1 -> FC2 without the h1 launch boundary
            if out is not None:
                return out
        h = _LinearReLU.apply(h, w1, b1, self)
        if w2 is None:  # the second layer from the branch parameters in place
            return self._heads_fc2(h)
        return torch.addmm(b2, h, w2.t())

    def _heads_counted(self, h, w1, b1, n_dev, n_fixed, cache):
        """forward_heads' device-counted heads: FC1 + ReLU as one GEMM over all n rows, or (n_fixed)
        a GEMM over the n_fixed live rows and rth_linear_relu_rows_upto over the counted rows
        behind them (usually none); then the second layer (+ the heads-cache scatter) over the
        counted rows only"""
        from ._lib import c_vp, call, lib, ptr, stream_ptr

        n, F = h.shape
        O = w1.shape[0]
        if n_fixed is None:
            h1 = _LinearReLU.apply(h, w1, b1, self)
        else:
            n_fixed = int(n_fixed)
            if not (0 < n_fixed <= n) or not h.is_contiguous():
                raise ValueError(f"forward_heads: n_fixed {n_fixed} outside (0, {n}] or features not contiguous")
            h1 = torch.empty((n, O), dtype=torch.float32, device=h.device)
            if w1.is_contiguous() and lib().rth_fc_x9_supported(n_fixed, O, F):
                # the x9 GEMM over the fixed rows, then its split-K reduce and the counted rows in one launch
                ws = _fc_workspace("rth_fc_x9", h.device, w1, n_fixed, O, F, self)
                call("rth_fc_x9_rows_upto", ptr(h), F, n_fixed, n, ptr(n_dev), ptr(w1), O, F, ptr(b1), ptr(h1), ptr(ws),
                     stream_ptr())
            else:  # (fixed rows not a multiple of 64: tiny actor counts) every counted row in HIP
                call("rth_linear_relu_rows_upto", ptr(h), F, 0, n, ptr(n_dev), ptr(w1), ptr(b1), F, O, ptr(h1), O,
                     stream_ptr())
        ps = self._head_params()[4:]
        A, H = ps[0].shape
        out = torch.empty((n, A + 1), dtype=torch.float32, device=h.device)
        arr = (c_vp * 4)(*[p.data_ptr() for p in ps])
        qc, qrows = cache if cache is not None else (None, None)
        if qc is not None and (qc.shape[1] != A + 1 or qrows.numel() < n or qrows.dtype != torch.int64):
            raise ValueError("forward_heads: heads cache of the wrong width or too few cache rows")
        call("rth_heads_fc2_upto", ptr(h1), h1.stride(0), n, ptr(n_dev), H, A, arr, ptr(out), ptr(qc), ptr(qrows),
             stream_ptr())
        return out

    def _convs(self):
        return [m for m in self.features if isinstance(m, nn.Conv2d)]

    def _torso_shapes(self, x_shape, u8):
        """per conv (None, rth_conv_shape or None), cached per (input shape, form, hip_conv)"""
        cache = self.__dict__.setdefault("_shape_cache", {})
        key = (tuple(x_shape), bool(u8), self.hip_conv)
        if key not in cache:
            cache[key] = self._conv_shapes(x_shape, u8)
        return cache[key]

    def pack_convs(self, u8=None, out=None, extra=()):
        """the HIP torso's packed conv weights (rth_conv_pack, fragment order) for the current
        parameters: [per conv: a device buffer, or None where MIOpen runs the layer].  Built
        for both conv1 input forms (f32 channels-last and uint8 stacks share conv2/conv3);
        `out` (a previous result) is refilled in place.  `extra`: further (shape, weight
        pointer, buffer pointer) jobs packed in the same launch (the learner's data-gradient
        kernels, shape.input | CONV_PACK_DGRAD)."""
        from . import _lib

        convs = self._convs()
        dev = convs[0].weight.device
        res = [] if out is None else out
        forms = [False, True] if u8 is None else [bool(u8)]
        jobs, keep, k = [], [], 0
        for form in forms:
            for li, (conv, (_, shape)) in enumerate(zip(convs, self._torso_shapes(self.input_shape, form))):
                if form and li > 0 and len(forms) == 2:
                    continue  # conv2 / conv3 are the same for both forms
                buf = None
                if shape is not None:
                    w = conv.weight.detach()
                    if not w.is_contiguous(memory_format=torch.channels_last):
                        w = w.contiguous(memory_format=torch.channels_last)
                        keep.append(w)
                    buf = res[k] if out is not None else torch.empty(
                        _lib.lib().rth_conv_packed_bytes(_lib.ctypes.byref(shape)) // 4, dtype=torch.float32,
                        device=dev)
                    jobs.append((shape, w.data_ptr(), buf.data_ptr()))
                if out is None:
                    res.append(buf)
                k += 1
        jobs.extend(extra)
        if jobs:  # one launch for the whole torso
            n = len(jobs)
            shapes = (_lib.ConvShape * n)(*[j[0] for j in jobs])
            ws = (_lib.c_vp * n)(*[j[1] for j in jobs])
            pks = (_lib.c_vp * n)(*[j[2] for j in jobs])
            _lib.call("rth_conv_pack_many", n, shapes, ws, pks, _lib.stream_ptr())
        return res

    @staticmethod
    def _packed_for(packed, li, u8):
        """packed buffer of conv li for the given conv1 input form (pack_convs layout: both
        forms [conv1 f32, conv2, conv3, conv1 u8]; one form [conv1, conv2, conv3])"""
        if li == 0 and u8 and len(packed) > 3:
            return packed[3]
        return packed[li]

    def _features_nhwc(self, x, rows=None, packed=None, n_dev=None):
        """the conv torso on channels-last activations: each Conv2d -> ReLU is one HIP
        implicit-GEMM launch with the bias and ReLU fused (rth_conv_bias_relu) where the
        geometry is built, else MIOpen + the rth_bias_relu pass; the last HIP conv writes its
        output NCHW (FC1 reads the reference's (C, H, W) flatten order); backward:
        rth_relu_bias_grad(_nchw) and MIOpen's data/weight gradients"""
        from . import _lib
        from .replay import FrameStacks

        if isinstance(x, FrameStacks) and (rows is not None or n_dev is not None or (
                torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()))):
            x = x.stacks()  # (frames in place is inference / the explicit learner pass only)
        u8 = x.dtype == torch.uint8
        if not u8 and not x.is_contiguous(memory_format=torch.channels_last):
            x = x.contiguous(memory_format=torch.channels_last)
        convs = self._convs()
        if getattr(self, "_ws", None) is None or self._ws[0].device != x.device:
            self._ws = [torch.zeros(_lib.lib().rth_relu_bias_grad_workspace(m.out_channels), dtype=torch.uint8,
                                    device=x.device) for m in convs]
        shapes = self._torso_shapes(x.shape[1:], u8)
        if packed is None and any(s is not None for _, s in shapes):
            packed = self.pack_convs(u8)
        if n_dev is not None:  # device-counted inference batch: every layer in rth_conv_bias_relu_upto
            from ._lib import call, ptr, stream_ptr

            if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
                raise RuntimeError("forward_heads(n_dev=...) is inference only (no autograd)")
            if any(sh is None for _, sh in shapes):
                raise ValueError("forward_heads(n_dev=...) needs every conv in rth_conv_bias_relu")
            n = rows.numel() if rows is not None else x.shape[0]
            for li, conv in enumerate(convs):
                shape = shapes[li][1]
                last = li == len(convs) - 1
                ho = (shape.hin - shape.kh) // shape.stride + 1
                wo = (shape.win - shape.kw) // shape.stride + 1
                y = torch.empty((n, shape.cout, ho, wo), dtype=torch.float32, device=x.device,
                                memory_format=torch.contiguous_format if last else torch.channels_last)
                call("rth_conv_bias_relu_upto", _lib.ctypes.byref(nchw_out(shape) if last else shape), ptr(x),
                     ptr(rows) if li == 0 else None, n, ptr(n_dev), ptr(self._packed_for(packed, li, u8)),
                     ptr(conv.bias), ptr(y), stream_ptr())
                x = y
            return x
        for li, (conv, ws) in enumerate(zip(convs, self._ws)):
            shape = shapes[li][1]
            if isinstance(x, FrameStacks):  # conv1 from the frame store (no autograd: checked above)
                from ._lib import call, ptr, stream_ptr

                if shape is None:
                    raise ValueError("frame-id batches need rth_conv_bias_relu's conv1 geometry")
                y = torch.empty((x.shape[0], shape.cout, (shape.hin - shape.kh) // shape.stride + 1,
                                 (shape.win - shape.kw) // shape.stride + 1), dtype=torch.float32, device=x.device,
                                memory_format=torch.channels_last)
                call("rth_conv1_frames_bias_relu", _lib.ctypes.byref(shape), ptr(x.store), ptr(x.ids), x.shape[0],
                     ptr(self._packed_for(packed, li, u8)), ptr(conv.bias), ptr(y), stream_ptr())
                x = y
                continue
            if shape is not None:
                pk = self._packed_for(packed, li, u8)
                last = li == len(convs) - 1 and li > 0  # the last conv writes NCHW (FC1's flatten order)
                x = _HipConvBiasReLU.apply(x, conv.weight, conv.bias, pk, nchw_out(shape) if last else shape,
                                           conv.stride, ws, rows if li == 0 else None)
            else:
                if x.dtype == torch.uint8 or (li == 0 and rows is not None):
                    raise ValueError("uint8 / row-indexed observations need rth_conv_bias_relu's conv1 geometry")
                x = _ConvBiasReLU.apply(x, conv.weight, conv.bias, conv.stride, ws)
        return x

    def _conv_shapes(self, x_shape, u8):
        """per conv: (None, rth_conv_shape or None when MIOpen runs it)"""
        from . import _lib

        out = []
        c, h, w = x_shape
        for li, conv in enumerate(m for m in self.features if isinstance(m, nn.Conv2d)):
            kind = _lib.CONV_U8_CHW if (u8 and li == 0) else _lib.CONV_F32_NHWC
            shp = _lib.ConvShape(kind, c, h, w, conv.out_channels, conv.kernel_size[0], conv.kernel_size[1],
                                 conv.stride[0])
            ok = (self.hip_conv and conv.stride[0] == conv.stride[1] and conv.padding == (0, 0)
                  and conv.dilation == (1, 1) and conv.groups == 1
                  and _lib.lib().rth_conv_supported(_lib.ctypes.byref(shp)) == 1)
            out.append((None, shp if ok else None))
            c, h, w = conv.out_channels, (h - conv.kernel_size[0]) // conv.stride[0] + 1, \
                (w - conv.kernel_size[1]) // conv.stride[1] + 1
        return out


class _MergeHeads(torch.autograd.Function):
    """(w1, b1, w2, b2) of the merged dueling heads from the eight branch parameters
    (rth_heads_merge) and their gradients back (rth_heads_split_grad)"""

    @staticmethod
    def forward(ctx, dims, *ps):
        from ._lib import c_vp, call, ptr, stream_ptr

        H, F, A, C, P = dims
        ps = [p.contiguous() for p in ps]
        o = dict(device=ps[0].device, dtype=torch.float32)
        w1, b1 = torch.empty(2 * H, F, **o), torch.empty(2 * H, **o)
        w2, b2 = torch.empty(A + 1, 2 * H, **o), torch.empty(A + 1, **o)
        arr = (c_vp * 8)(*[p.data_ptr() for p in ps])
        call("rth_heads_merge", arr, H, F, A, C, P, ptr(w1), ptr(b1), ptr(w2), ptr(b2), stream_ptr())
        ctx.dims = dims
        ctx.shapes = [p.shape for p in ps]
        return w1, b1, w2, b2

    @staticmethod
    def backward(ctx, gw1, gb1, gw2, gb2):
        from ._lib import c_vp, call, ptr, stream_ptr

        H, F, A, C, P = ctx.dims
        outs = [gw1, gb1, gw2, gb2]
        shapes = [(2 * H, F), (2 * H,), (A + 1, 2 * H), (A + 1,)]
        ref = next(g for g in outs if g is not None)
        outs = [torch.zeros(s, device=ref.device) if g is None else g.contiguous() for g, s in zip(outs, shapes)]
        grads = [torch.empty(s, device=ref.device) for s in ctx.shapes]
        arr = (c_vp * 8)(*[g.data_ptr() for g in grads])
        call("rth_heads_split_grad", ptr(outs[0]), ptr(outs[1]), ptr(outs[2]), ptr(outs[3]), H, F, A, C, P, arr,
             stream_ptr())
        return (None, *grads)


# FC1 + bias + ReLU of every forward -- the actors' (256 rows at Pong, 2,048 at Breakout), the
# target pass's (512) and, since r06, the learner's [s0; s1] (1,024) -- runs on rth_fc_x9 (the
# exact-split bf16 MFMA: every product exact, fixed-order split-K) where the shape is built
# (rows % 64, N % 128, K % 32), else on hipBLASLt's GEMM with the bias+ReLU epilogue.  The
# learner's forward moved off hipBLASLt for accuracy: its MT32x64x64 kernel
# sums each output as one 3,136-term fp32 chain, 4.4x the reference CPU GEMM's local error,
# which made the end-to-end |td| 2.1x the reference fp32 run's distance from the exact |td|; on
# x9 it is 1.1x.  Cost in the loop: 0.516 -> 0.520 ms/step (interleaved, 3 rounds,
# profiles/r06/ab_log.txt).
_FC_WS = {}


# FC1_HEADS -- FC1's split-K reduce and FC2 in one launch (rth_fc1_heads) wherever the heads are
# computed without autograd: the target pass and the learner's forward (r06); tests patch it
FC1_HEADS = True


def _fc_workspace(fn, device, w, M, N, K, owner=None):
    """the split-K workspace of fn for (M, N, K), owned by the network that runs it (`owner`: its
    workspaces live and die with it -- a module-level cache keyed by pointers would hand a later
    network, allocated at a freed one's addresses, buffers from a released graph pool) and keyed
    by the launching stream: the same network may run the same shape on two streams at once (the
    target network's B-row pass: the learner's own after a target sync on the learner stream,
    the next batch's on the actor stream), and a shared workspace would mix the two launches'
    split-K partials"""
    from ._lib import lib, stream_ptr

    cache = owner.__dict__.setdefault("_fc_ws", {}) if owner is not None else _FC_WS
    key = (device, w.data_ptr(), M, N, K, fn, stream_ptr())
    ws = cache.get(key)
    if ws is None:
        ws = cache[key] = torch.empty(max(getattr(lib(), fn + "_workspace")(M, N, K), 16) // 4, dtype=torch.float32,
                                      device=device)
    return ws


def fc1_relu(x, w, b, out=None, owner=None):
    """relu(x @ w.T + b) (FC1 of both dueling branches): rth_fc_x9 where built for the shape,
    else one hipBLASLt GEMM with the bias+ReLU epilogue.  The split-K workspace is keyed by the
    weight storage, so two networks (the actors', the target's, the learner's -- on different
    streams) never share one"""
    M, K = x.shape
    N = w.shape[0]
    if x.is_cuda and x.stride(1) == 1 and w.is_contiguous():
        from ._lib import call, lib, ptr, stream_ptr

        if lib().rth_fc_x9_supported(M, N, K):
            y = out if out is not None else torch.empty((M, N), dtype=torch.float32, device=x.device)
            ws = _fc_workspace("rth_fc_x9", x.device, w, M, N, K, owner)
            call("rth_fc_x9", ptr(x), x.stride(0), M, ptr(w), N, K, ptr(b), 1, ptr(y), ptr(ws), stream_ptr())
            return y
    if out is not None:
        return torch._addmm_activation(b, x, w.t(), out=out)
    return torch._addmm_activation(b, x, w.t())


class _LinearReLU(torch.autograd.Function):
    """relu(x @ w.T + b) as one fc1_relu launch (rth_fc_x9, or hipBLASLt's GEMM with a bias+ReLU
    epilogue: torch._addmm_activation has no autograd formula of its own); the backward is the
    one autograd derives for linear -> relu (threshold on the output, addmm grads)."""

    @staticmethod
    def forward(ctx, x, w, b, owner=None):
        out = fc1_relu(x, w, b, owner=owner)
        ctx.save_for_backward(x, w, out)
        return out

    @staticmethod
    def backward(ctx, g):
        x, w, out = ctx.saved_tensors
        g = torch.ops.aten.threshold_backward(g, out, 0)
        gx = g.mm(w) if ctx.needs_input_grad[0] else None
        gw = g.t().mm(x) if ctx.needs_input_grad[1] else None
        gb = g.sum(0) if ctx.needs_input_grad[2] else None
        return gx, gw, gb, None


class _ConvBiasReLU(torch.autograd.Function):
    """relu(conv2d(x, w) + b) on channels-last fp32: MIOpen convolution without bias, then
    rth_bias_relu in place; backward: rth_relu_bias_grad (mask + bias gradient in one pass)
    and MIOpen's data/weight gradients (dqn_model.py:14-20)."""

    @staticmethod
    def forward(ctx, x, w, b, stride, ws):
        from ._lib import call, ptr, stream_ptr

        y = torch.ops.aten.convolution(x, w, None, list(stride), [0, 0], [1, 1], False, [0, 0], 1)
        if not y.is_contiguous(memory_format=torch.channels_last):
            y = y.contiguous(memory_format=torch.channels_last)
        n, c, h, wd = y.shape
        call("rth_bias_relu", ptr(y), ptr(b), n * h * wd, c, stream_ptr())
        ctx.save_for_backward(x, w, y)
        ctx.stride, ctx.ws = list(stride), ws
        return y

    @staticmethod
    def backward(ctx, g):
        from ._lib import call, ptr, stream_ptr

        x, w, y = ctx.saved_tensors
        if not g.is_contiguous(memory_format=torch.channels_last):
            g = g.contiguous(memory_format=torch.channels_last)
        gy = torch.empty_like(y)
        n, c, h, wd = y.shape
        db = torch.empty(c, dtype=y.dtype, device=y.device)
        call("rth_relu_bias_grad", ptr(g), ptr(y), ptr(gy), ptr(db), ptr(ctx.ws), n * h * wd, c, stream_ptr())
        gx, gw, _ = torch.ops.aten.convolution_backward(gy, x, w, None, ctx.stride, [0, 0], [1, 1], False, [0, 0], 1,
                                                        [ctx.needs_input_grad[0], ctx.needs_input_grad[1], False])
        return gx, gw, db, None, None


_WGRAD_WS = {}


def _wgrad_workspace(shape, device):
    """rth_conv_relu_wgrad's partial-sum workspace (one per device; backward passes on a
    device run in stream order)"""
    from ._lib import ctypes, lib

    key = (device, shape.input, shape.cin, shape.cout)
    ws = _WGRAD_WS.get(key)
    if ws is None:
        nbytes = lib().rth_conv_wgrad_workspace(ctypes.byref(shape))
        ws = _WGRAD_WS[key] = torch.empty(max(nbytes, 16) // 4, dtype=torch.float32, device=device)
    return ws


class _HipConvBiasReLU(torch.autograd.Function):
    """relu(conv2d(x, w) + b) as one rth_conv_bias_relu launch (conv.hip); x channels-last
    fp32, or uint8 CHW frame stacks (optionally through a row index) for the first layer.
    Backward as _ConvBiasReLU: rth_relu_bias_grad + MIOpen data/weight gradients (a uint8
    input is widened to the f32 channels-last batch it stands for)."""

    @staticmethod
    def forward(ctx, x, w, b, packed, shape, stride, ws, rows):
        from ._lib import call, ctypes, ptr, stream_ptr

        from ._lib import CONV_OUT_NCHW

        n = rows.numel() if rows is not None else x.shape[0]
        ho = (shape.hin - shape.kh) // shape.stride + 1
        wo = (shape.win - shape.kw) // shape.stride + 1
        nchw = bool(shape.input & CONV_OUT_NCHW)
        y = torch.empty((n, shape.cout, ho, wo), dtype=torch.float32, device=x.device,
                        memory_format=torch.contiguous_format if nchw else torch.channels_last)
        call("rth_conv_bias_relu", ctypes.byref(shape), ptr(x), ptr(rows), n, ptr(packed), ptr(b), ptr(y),
             stream_ptr())
        ctx.nchw = nchw
        ctx.save_for_backward(x, w, y, rows)
        ctx.stride, ctx.ws, ctx.shape = list(stride), ws, shape
        ctx.wgrad_ws = None
        if x.dtype == torch.uint8 and ctx.needs_input_grad[1]:
            ctx.wgrad_ws = _wgrad_workspace(shape, x.device)
        return y

    @staticmethod
    def backward(ctx, g):
        from ._lib import call, ptr, stream_ptr

        x, w, y, rows = ctx.saved_tensors
        fmt = torch.contiguous_format if ctx.nchw else torch.channels_last
        if not g.is_contiguous(memory_format=fmt):
            g = g.contiguous(memory_format=fmt)
        if x.dtype == torch.uint8 and ctx.wgrad_ws is not None:
            # conv1 on uint8 stacks: ReLU mask + weight and bias gradients in one HIP pass
            # (rth_conv_relu_wgrad), straight from the stacks
            from ._lib import ctypes

            gw = torch.empty(w.shape, dtype=w.dtype, device=w.device, memory_format=torch.channels_last)
            db = torch.empty(w.shape[0], dtype=w.dtype, device=w.device)
            n = y.shape[0]
            call("rth_conv_relu_wgrad", ctypes.byref(ctx.shape), ptr(x), ptr(rows), n, ptr(g), ptr(y), ptr(gw),
                 ptr(db), ptr(ctx.wgrad_ws), stream_ptr())
            return None, gw if ctx.needs_input_grad[1] else None, db, None, None, None, None, None
        if not w.is_contiguous(memory_format=torch.channels_last):
            w = w.contiguous(memory_format=torch.channels_last)
        if x.dtype == torch.uint8:
            x = (x if rows is None else x[rows]).float().contiguous(memory_format=torch.channels_last)
        n, c, h, wd = y.shape
        gy = torch.empty((n, c, h, wd), dtype=y.dtype, device=y.device, memory_format=torch.channels_last)
        db = torch.empty(c, dtype=y.dtype, device=y.device)
        if ctx.nchw:  # mask + bias gradient from the NCHW output, gy written channels-last
            call("rth_relu_bias_grad_nchw", ptr(g), ptr(y), ptr(gy), ptr(db), ptr(ctx.ws), n, c, h * wd, stream_ptr())
        else:
            call("rth_relu_bias_grad", ptr(g), ptr(y), ptr(gy), ptr(db), ptr(ctx.ws), n * h * wd, c, stream_ptr())
        need_x = ctx.needs_input_grad[0]
        gx, gw, _ = torch.ops.aten.convolution_backward(gy, x, w, None, ctx.stride, [0, 0], [1, 1], False, [0, 0], 1,
                                                        [need_x, ctx.needs_input_grad[1], False])
        return gx, gw, db, None, None, None, None, None


class MLP_DQNNetwork(nn.Module):
    """dqn_model.py:59-71: obs (D,) -> Q[A] (CartPole)."""

    def __init__(self, obs_shape, num_actions):
        super().__init__()
        self.nn = nn.Sequential(nn.Linear(obs_shape[0], 128), nn.ReLU(inplace=True), nn.Linear(128, 128),
                                nn.ReLU(inplace=True), nn.Linear(128, num_actions))

    def forward(self, x):
        return self.nn(x)


def make_q_network(obs_shape, num_actions, dueling=True):
    """generate_dqn_network (dqn_model.py:74-83): conv net for 3-D observations, MLP otherwise"""
    if len(obs_shape) == 3:
        return DQNNetwork(obs_shape, num_actions, dueling=dueling)
    return MLP_DQNNetwork(obs_shape, num_actions)


def default_models(obs_shape, num_actions, dueling=True, learning_rate=5e-5, adam_epsilon=1e-8, fused_adam=True):
    """generate_dqn_default_models (dqn_model.py:86-99): online net, target net, Adam."""
    q = make_q_network(obs_shape, num_actions, dueling)
    tq = make_q_network(obs_shape, num_actions, dueling)
    return {"q_network": q, "target_q_network": tq, "learning_rate": learning_rate, "adam_epsilon": adam_epsilon,
            "fused_adam": fused_adam}
