"""Development aid (r06): are the actors' device-counted FC1 tail rows deterministic while the
learner's x9 FC1 runs on another stream?  Stream A repeats the actors' counted FC1 (x9 over the
256 fixed rows + the tail row 256 in the reduce launch, then the in-place second layer) on fixed
inputs; stream B repeats the learner's 1,024-row x9 FC1.  Every repetition's tail row is kept;
all must equal the first.  usage: diag_tail_concurrency.py [reps] [rows|x9] [noB]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reth_amd._lib import c_vp, call, lib, ptr  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
form = sys.argv[2] if len(sys.argv) > 2 else "x9"
use_b = "noB" not in sys.argv[3:]
bmode = next((a[2:] for a in sys.argv[3:] if a.startswith("b=")), "x9")  # B's kernel: x9 | f32 | mm | copy
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(1)
N, F, O, A = 256, 3136, 512, 6
h = torch.rand((2 * N, F), device=dev, generator=g)
w1 = (torch.rand((O, F), device=dev, generator=g) - 0.5) * 0.05
b1 = (torch.rand(O, device=dev, generator=g) - 0.5) * 0.1
wa2 = (torch.rand((A, O // 2), device=dev, generator=g) - 0.5) * 0.1
wv2 = (torch.rand((1, O // 2), device=dev, generator=g) - 0.5) * 0.1
ba2 = torch.zeros(A, device=dev)
bv2 = torch.zeros(1, device=dev)
n_dev = torch.tensor([N + 1], dtype=torch.int64, device=dev)
h1 = torch.zeros((2 * N, O), device=dev)
out = torch.zeros((2 * N, A + 1), device=dev)
ws = torch.empty(max(lib().rth_fc_x9_workspace(N, O, F), 16) // 4, device=dev)
arr = (c_vp * 4)(*[p.data_ptr() for p in (wa2, wv2, ba2, bv2)])
hist_h1 = torch.zeros((reps, O), device=dev)
hist_q = torch.zeros((reps, A + 1), device=dev)
# the learner's FC1 on stream B
xl = torch.rand((4 * N, F), device=dev, generator=g)
yl = torch.empty((4 * N, O), device=dev)
wsl = torch.empty(max(lib().rth_fc_x9_workspace(4 * N, O, F), lib().rth_fc_f32_workspace(4 * N, O, F), 16) // 4,
                  device=dev)
big = torch.empty(64 << 20, device=dev)
w1b = w1.clone() if "sepw" in sys.argv[3:] else w1  # B's x9 on its own copy of the weights
hist_pre = torch.zeros((reps, O), device=dev)
blib = next((a[5:] for a in sys.argv[3:] if a.startswith("blib=")), None)  # B's rth_fc_x9 from another build
if blib:
    import ctypes
    bl = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), blib))
    bl.rth_fc_x9.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                             ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p]
hog_bad = torch.zeros(1, dtype=torch.int32, device=dev)
if form.startswith("probe"):
    import ctypes
    rp = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "probes",
                                  "librows_probe_nopk.so" if "nopk" in sys.argv[3:] else "librows_probe.so"))
    rp.rows_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                              ctypes.c_void_p, ctypes.c_void_p]
    rp.rows_probe_mod.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    rp.rows_probe_ex.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
if bmode.startswith("hog"):
    import ctypes
    hog = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "probes", "liblds_hog.so"))
    hog.lds_hog.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]
torch.cuda.synchronize()
sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
for i in range(reps):
    with torch.cuda.stream(sa):
        h1[N:].fill_(float("nan"))  # the tail row must be written by this repetition
        if form == "x9":
            call("rth_fc_x9_rows_upto", ptr(h), F, N, 2 * N, ptr(n_dev), ptr(w1), O, F, ptr(b1), ptr(h1), ptr(ws),
                 sa.cuda_stream)
        elif form.startswith("probe") and int(form[5:]) >= 9:
            assert rp.rows_probe_mod(int(form[5:]), h.data_ptr(), N, n_dev.data_ptr(), w1.data_ptr(), b1.data_ptr(), F, O,
                                     h1.data_ptr(), sa.cuda_stream) == 0
        elif form.startswith("probe") and int(form[5:]) >= 3:
            assert rp.rows_probe_ex(int(form[5:]), h.data_ptr(), N, n_dev.data_ptr(), w1.data_ptr(), b1.data_ptr(), F, O,
                                    h1.data_ptr(), sa.cuda_stream) == 0
        elif form.startswith("probe"):
            assert rp.rows_probe(int(form[5:]), h[N].data_ptr(), w1.data_ptr(), b1.data_ptr(), F, O, h1[N].data_ptr(),
                                 sa.cuda_stream) == 0
        else:
            call("rth_linear_relu_rows_upto", ptr(h), F, 0, 2 * N, ptr(n_dev), ptr(w1), ptr(b1), F, O, ptr(h1), O,
                 sa.cuda_stream)
        hist_pre[i].copy_(h1[N])
        call("rth_heads_fc2_upto", ptr(h1), O, 2 * N, ptr(n_dev), O // 2, A, arr, ptr(out), None, None, sa.cuda_stream)
        hist_h1[i].copy_(h1[N])
        hist_q[i].copy_(out[N])
    if use_b:
        with torch.cuda.stream(sb):
            for _ in range(2):
                if bmode == "x9" and blib:
                    assert bl.rth_fc_x9(xl.data_ptr(), F, 4 * N, w1b.data_ptr(), O, F, b1.data_ptr(), 1, yl.data_ptr(),
                                        wsl.data_ptr(), sb.cuda_stream) == 0
                elif bmode == "x9":
                    call("rth_fc_x9", ptr(xl), F, 4 * N, ptr(w1b), O, F, ptr(b1), 1, ptr(yl), ptr(wsl), sb.cuda_stream)
                elif bmode == "f32":
                    call("rth_fc_f32", ptr(xl), F, 4 * N, ptr(w1), O, F, ptr(b1), 1, ptr(yl), ptr(wsl), sb.cuda_stream)
                elif bmode == "mm":
                    torch.mm(xl, w1.t(), out=yl)
                elif bmode.startswith("hog"):
                    assert hog.lds_hog(int(bmode[3:]), 256, 40, 7, hog_bad.data_ptr(), sb.cuda_stream) == 0
                else:
                    big.mul_(1.0000001)
torch.cuda.synchronize()
bad_h1 = [i for i in range(reps) if not torch.equal(hist_h1[i], hist_h1[0])]
bad_q = [i for i in range(reps) if not torch.equal(hist_q[i], hist_q[0])]
late = [i for i in range(reps) if not torch.equal(hist_pre[i], hist_h1[i])]
print("h1 row changed between the rows launch and the heads launch in reps", late[:10], flush=True)
ref = torch.relu(h[N].double() @ w1.double().t() + b1.double())
print(form, ("B=" + bmode) if use_b else "noB", "reps", reps, "tail h1 differing reps", len(bad_h1), bad_h1[:10],
      "heads differing reps", len(bad_q), bad_q[:10], "h1[0] max err vs fp64", float((hist_h1[0].double() - ref).abs().max()),
      "hog bad reads", int(hog_bad.item()), flush=True)
for i in bad_h1[:3]:
    d = (hist_h1[i] - hist_h1[0]).abs()
    cols = torch.nonzero(d > 0).flatten()
    print("  rep", i, "columns differing", cols.numel(), cols[:24].tolist(), "max", float(d.max()), flush=True)
