"""Development aid (r06): the Ape-X loop graph-replayed twice with the same seed (lr = 0, Pong
size, after a learning run as test_scale_gpu does) -- do two graph runs agree with each other
and with the eager run?  The tree's root sum per iteration.  usage: diag_graph_race.py [overlap 0/1]"""
import gc
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reth_amd.apex import ApexConfig, ApexDQN  # noqa: E402

overlap = (sys.argv[1] != "0") if len(sys.argv) > 1 else True
sync = "sync" in sys.argv[2:]  # synchronize after every iteration
nopub = "nopub" in sys.argv[2:]  # no weights publish to the actors within the run
if "blas" in sys.argv[2:]:  # the learner's FC1 forward on hipBLASLt
    from reth_amd import fused_learner
    fused_learner.fc1_relu = lambda x, w, b, out=None, owner=None: torch._addmm_activation(b, x, w.t())
if "notgt" in sys.argv[2:]:  # no target pass precomputed on the actor stream: every learner step "full"
    _orig_capture = ApexDQN._capture_graphs

    class _NoGraph:
        def replay(self):
            pass

    def _capture_graphs(self, solver, slots):
        _orig_capture(self, solver, slots)
        self._graphs["tgt"] = [_NoGraph(), _NoGraph()]

    ApexDQN._capture_graphs = _capture_graphs
    _orig_it = ApexDQN._iteration_graph_overlap

    def _it(self):
        _orig_it(self)
        self._q1t_ready = [False, False]

    ApexDQN._iteration_graph_overlap = _it
if "dep1" in sys.argv[2:]:  # the learner waits for the whole actor block of its iteration
    _orig_lr = ApexDQN._learner_replay

    def _lr(self, v):
        torch.cuda.current_stream(self.device).wait_stream(self._stream)
        _orig_lr(self, v)

    ApexDQN._learner_replay = _lr
if "c1" in sys.argv[2:]:  # the learner waits for the actor graph of its iteration, not the append
    _orig_lr1 = ApexDQN._learner_replay

    def _lr1(self, v):
        if getattr(self, "_ev_c1", None) is not None:
            torch.cuda.current_stream(self.device).wait_event(self._ev_c1)
        _orig_lr1(self, v)

    ApexDQN._learner_replay = _lr1
c1 = "c1" in sys.argv[2:]
dep2 = "dep2" in sys.argv[2:]  # the sample-ahead (and target pass) wait for the learner
if "wx9" in sys.argv[2:]:  # conv2 / conv3 weight gradients on rth_conv_wgrad_x9 instead of MIOpen
    from reth_amd import fused_learner as _fl
    _fl.HIP_WGRAD = "x9"
if "wsfresh" in sys.argv[2:]:  # the learner's FC1 workspace allocated eagerly (default pool), one per shape
    from reth_amd import fused_learner as _fl2
    from reth_amd import model as _m
    _WS = {}

    def _fc1(x, w, b, out=None, owner=None):
        from reth_amd._lib import call, lib, ptr, stream_ptr
        M, K = x.shape
        N = w.shape[0]
        key = (M, N, K)
        if key not in _WS:
            assert not torch.cuda.is_current_stream_capturing()
            _WS[key] = torch.empty(max(lib().rth_fc_x9_workspace(M, N, K), 16) // 4, dtype=torch.float32, device=x.device)
        y = torch.empty((M, N), dtype=torch.float32, device=x.device)
        call("rth_fc_x9", ptr(x), x.stride(0), M, ptr(w), N, K, ptr(b), 1, ptr(y), ptr(_WS[key]), stream_ptr())
        return y

    _fl2.fc1_relu = _fc1
if "actrows" in sys.argv[2:]:  # the actors' FC1 on rth_linear_relu_rows_upto (no x9 GEMM in the actor graph)
    from reth_amd import _lib as _L
    _orig_lib = _L.lib

    class _Proxy:
        def __init__(self, real):
            self._real = real

        def __getattr__(self, k):
            if k == "rth_fc_x9_supported":
                return lambda M, N, K: 0 if M == 256 else self._real.rth_fc_x9_supported(M, N, K)
            return getattr(self._real, k)

    _L.lib = lambda: _Proxy(_orig_lib())
dev = torch.device("cuda", 0)
# device-side history of the actors' first tail rows (features and heads), one entry per actor step
from reth_amd.model import DQNNetwork  # noqa: E402
_orig_hc = DQNNetwork._heads_counted
HIST = {}


def _hc(self, h, w1, b1, n_dev, n_fixed, cache):
    out = _orig_hc(self, h, w1, b1, n_dev, n_fixed, cache)
    st = HIST.get("cur")
    if st is not None and h.shape[0] >= 260:
        c, hf, hq = st
        hf.index_copy_(0, c, h[256:260].reshape(1, -1))
        hq.index_copy_(0, c, out[256:260].reshape(1, -1))
        c.add_(1)
    return out


DQNNetwork._heads_counted = _hc
kw = dict(n_actors=256, num_actions=6, capacity=1_000_000)
prefill = (1_000_000 - 256 * 10) // 4


RUNS = []
HRUNS = []
ARUNS = []


def run(graph, seed=4, lr=0.0, iters=14, pre=prefill):
    ax = ApexDQN(ApexConfig(batch_size=512, hip_graph=graph, seed=seed, learning_rate=lr, overlap=overlap,
                            send_weights_interval=10 ** 6 if nopub else 10, **kw), device=dev)
    ax.prefill(pre)
    HIST["cur"] = (torch.zeros(1, dtype=torch.int64, device=dev), torch.zeros(64, 4 * 3136, device=dev),
                   torch.zeros(64, 4 * 7, device=dev))
    HRUNS.append(HIST["cur"])
    trace = []
    _orig_up = ax.replay.update_priorities

    def _up(indices, td_abs, *a, **k):
        if ax._graphs is None:  # eager: everything on one stream
            trace.append((indices.clone(), td_abs.clone()))
        return _orig_up(indices, td_abs, *a, **k)

    _orig_lr = ax._learner_replay
    _orig_lh = ax._learner_host

    def _lr(v):
        ax._diag_v = v
        return _orig_lr(v)

    def _lh():
        v = getattr(ax, "_diag_v", None)
        if v is not None:  # graph mode: cloned on the learner stream, right behind the learner block
            trace.append((ax.loader._slots[v[-1]][1].clone(), ax._graphs["learn_td"][v].clone()))
            ax._diag_v = None
        return _orig_lh()

    ax._learner_replay = _lr
    ax._learner_host = _lh

    ax.replay.update_priorities = _up
    atrace = []
    _orig_ap = ax.actors.append

    def _ap(replay, td, rows=None, *a, **k):
        atrace.append((td.clone(), None if rows is None else torch.cat([rows.a.double().flatten(), rows.r.double().flatten(),
                                                                          rows.done.double().flatten(),
                                                                          ax.actors.frames[rows.s0].sum(dim=(1, 2, 3)).double(),
                                                                          ax.actors.frames[rows.s1].sum(dim=(1, 2, 3)).double()]),
                       None if rows is None else (ax.actors.qcache[rows.s0].clone(), ax.actors.qcache[rows.s1].clone(),
                                                  rows.s0.clone(), rows.s1.clone(), ax.actors.hx.clone(),
                                                  ax.actors.n_ext.clone())))
        return _orig_ap(replay, td, rows, *a, **k)

    ax.actors.append = _ap
    ARUNS.append(atrace)
    RUNS.append(trace)
    if c1:
        _orig_append = ax.actors.append

        def _append(*a, **k):
            if ax._graphs is not None:
                ax._ev_c1 = torch.cuda.Event()
                ax._ev_c1.record(torch.cuda.current_stream(dev))
            return _orig_append(*a, **k)

        ax.actors.append = _append
    if dep2:
        _orig_issue = ax.loader.issue

        def _issue():
            if hasattr(ax, "_stream_b"):
                torch.cuda.current_stream(dev).wait_stream(ax._stream_b)
            return _orig_issue()

        ax.loader.issue = _issue
    rec = []
    for _ in range(iters):
        ax.iteration()
        if sync:
            torch.cuda.synchronize()
            rec.append(float(ax.replay.tree.export()[0][0]))
    torch.cuda.synchronize()
    from reth_amd.replay import tree_update_timeouts
    print("tree update timeouts", tree_update_timeouts(), flush=True)
    s, m, v = ax.replay.tree.export()
    rec.append((float(s[0]), float(s.double().sum()), float(v.double().sum())))
    ax.close()
    del ax
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return rec


first = run(True, seed=3, lr=1e-4, iters=30, pre=1_000_000 - 256 * 10)  # the test's learning run
eager = run(False)
g1 = run(True)
g2 = run(True)
for k, (e, a, b) in enumerate(zip(eager, g1, g2)):
    print(k, f"eager {e!r} graph1 {a!r} graph2 {b!r}", "g1==e" if a == e else "g1!=e", "g2==e" if b == e else "g2!=e",
          flush=True)
def _cmp(name, r):
    e = RUNS[1]
    for i, ((ie, te), (ig, tg)) in enumerate(zip(e, r)):
        if not torch.equal(ie, ig):
            print(name, "first idx difference at update", i, "rows", int((ie != ig).sum()), flush=True)
            return
        if not torch.equal(te, tg):
            d = (te - tg).abs()
            print(name, "first td difference at update", i, "rows", int((d > 0).sum()), "max", float(d.max()),
                  "rows idx", torch.nonzero(d > 0).flatten()[:16].tolist(), flush=True)
            return
    print(name, "all", len(e), "updates equal", flush=True)


def _acmp(name, r):
    e = ARUNS[1]
    for i, ((te, re_, xe), (tg, rg, xg)) in enumerate(zip(e, r)):
        if re_ is not None and rg is not None and not torch.equal(re_, rg):
            print(name, "first actor row difference at append", i, flush=True)
            return
        if not torch.equal(te, tg):
            d = (te - tg).abs()
            print(name, "first actor td difference at append", i, "rows", int((d > 0).sum()), "max", float(d.max()), flush=True)
            bad = torch.nonzero(d > 0).flatten().tolist()
            q0e, q1e, s0, s1, hxe, ne = xe
            q0g, q1g, _, _, hxg, ng = xg
            print("  rows", bad, "s0", s0[bad].tolist(), "s1", s1[bad].tolist(), "n_ext", ne.tolist(), ng.tolist(),
                  "hx equal", torch.equal(hxe, hxg), flush=True)
            for b in bad:
                print("  q(s0) eager", q0e[b].tolist(), "graph", q0g[b].tolist(), flush=True)
                print("  q(s1) eager", q1e[b].tolist(), "graph", q1g[b].tolist(), flush=True)
                sb = int(s1[b])
                print("  s1 stack in hx at", torch.nonzero(hxe == sb).flatten().tolist(), "s0 stack at",
                      torch.nonzero(hxe == int(s0[b])).flatten().tolist(), flush=True)
            n_diff = [(j, int((te2 - tg2).abs().gt(0).sum())) for j, ((te2, _, _), (tg2, _, _)) in enumerate(zip(e, r))]
            print("  per-append differing td rows", n_diff, flush=True)
            return
    print(name, "all", len(e), "appends equal", flush=True)


def _hcmp(name, r):
    c, hf, hq = HRUNS[1]
    c2, hf2, hq2 = r
    n = min(int(c), int(c2))
    print(name, "tail-row records", int(c), int(c2), flush=True)
    for i in range(n):
        fe = torch.equal(hf[i], hf2[i])
        qe = torch.equal(hq[i], hq2[i])
        if not (fe and qe):
            df = (hf[i] - hf2[i]).abs().view(4, -1)
            dq = (hq[i] - hq2[i]).abs().view(4, -1)
            print("  step", i, "features equal", fe, "heads equal", qe, "feature max diff per row",
                  df.max(dim=1).values.tolist(), "heads max diff per row", dq.max(dim=1).values.tolist(), flush=True)
            if not fe:
                nz = torch.nonzero(df[0] > 0).flatten()
                print("  row 256 differing features", nz.numel(), "first", nz[:20].tolist(), flush=True)


_hcmp("graph1", HRUNS[2])
_hcmp("graph2", HRUNS[3])
_acmp("graph1", ARUNS[2])
_acmp("graph2", ARUNS[3])
_cmp("graph1", RUNS[2])
_cmp("graph2", RUNS[3])
print("overlap", overlap, "args", sys.argv[2:])
