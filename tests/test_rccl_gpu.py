"""RCCL (torch.distributed "nccl" on ROCm) through the data-parallel learner's code path on
the one-GPU box: a one-rank process group with the gradient all-reduce forced on
(ApexConfig.dp_hook=True).  The captured learner is then cut at its two gradient buckets and the
heads' bucket is all-reduced on a side stream while the conv backward replays, the conv bucket
on the learner stream, exactly as at N > 1 (ApexDQN._learner_replay); averaging over one rank is
the identity, so the parameters must be bit-identical to the unhooked loop's.  The driver's
N = 2 / 4 / 8 runs are the first with more ranks (one GPU per rank); this pins the RCCL calls,
their streams and the graph cuts before them.  The RCCL work runs in a child process that
reports each stage, so a failure names the stage (process-group teardown included)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

CHILD = r'''
import json, os, sys
sys.path.insert(0, sys.argv[1])
# a run-to-run deterministic learner (the default weight gradients, rth_conv_wgrad_f32: MIOpen's
# solvers differ in the last bits run to run), so the hooked and the plain run can be compared
import torch
import torch.distributed as dist
from reth_amd import fused_learner
from reth_amd.apex import ApexConfig, ApexDQN
assert fused_learner.HIP_WGRAD == "f32"

def say(**kw):
    print("STAGE " + json.dumps(kw), flush=True)

dev = torch.device("cuda:0")

def run(dp_hook, iters=40, keep=False, probe=False):
    cfg = ApexConfig(n_actors=16, capacity=2048, batch_size=64, sample_start=128, seed=4, hip_graph=True,
                     send_weights_interval=3, recv_weights_interval=4, update_target_interval=7, dp_hook=dp_hook,
                     extra={"probe_conv2": True} if probe else {})
    ax = ApexDQN(cfg, device=dev, rank=0, world=1)
    tags = []
    ax.conv_probe = tags.append if probe else None
    for _ in range(iters):
        ax.iteration()
    torch.cuda.synchronize()
    parts = sorted({len(v) for v in ax._graphs["learn"].values()}) if ax._graphs else []
    params = torch.cat([p.detach().flatten() for p in ax.solver._params]).cpu()
    if keep:  # the captured graphs, the side streams and the bucket buffers stay alive
        return params, parts, ax
    ax.close()
    return params, parts, None

dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + sys.argv[2], rank=0, world_size=1)
say(stage="init", backend=dist.get_backend())
t = torch.arange(8, dtype=torch.float32, device=dev)
dist.all_reduce(t)
torch.cuda.synchronize()
say(stage="all_reduce", ok=bool(torch.equal(t.cpu(), torch.arange(8, dtype=torch.float32))))
mode = sys.argv[3]
if mode == "probe":  # the bench's probe copies cut at buckets AND probed launches: no empty part
    import warnings
    with warnings.catch_warnings(record=True) as wl:
        warnings.simplefilter("always")
        probed, parts, _ = run(True, probe=True)
    plain, _, _ = run(False)
    say(stage="probe", parts=parts, equal=bool(torch.equal(probed, plain)),
        empty=sum("CUDA Graph is empty" in str(w.message) for w in wl))
    os._exit(0)
hooked, parts, alive = run(True, keep=mode != "keep")
say(stage="hooked", parts=parts)
plain, parts0, _ = run(False)
say(stage="plain", parts=parts0, equal=bool(torch.equal(hooked, plain)))
if mode == "keep":
    os._exit(0)
if mode == "destroy_alive":  # the group destroyed while the hooked loop's graphs are still alive
    for _ in range(3):  # the comm stream has just carried RCCL work
        alive.iteration()
    dist.destroy_process_group()
    say(stage="destroyed")
    import gc
    alive.close()
    del alive
    gc.collect()
    torch.cuda.synchronize()
    say(stage="closed")
else:  # "shutdown": bench.py's teardown (reth_amd.dist.shutdown: graphs released, then the group)
    from reth_amd.dist import shutdown
    alive.iteration()
    shutdown(alive)
    say(stage="destroyed", initialized=dist.is_initialized())
# a normal interpreter exit: HIP / RCCL / graph destructors run
'''


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _child(teardown):
    import torch

    if torch.cuda.is_initialized():  # hand the suite's cached device memory back before the child starts
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", CHILD, root, str(_free_port()), teardown], capture_output=True,
                       text=True, timeout=200)
    stages = {}
    for line in p.stdout.splitlines():
        if line.startswith("STAGE "):
            d = json.loads(line[6:])
            stages[d.pop("stage")] = d
    err = p.stderr
    hits = [ln for ln in err.splitlines() if "error" in ln.lower() or "what()" in ln][:8]
    return p.returncode, stages, "\n".join(hits) + "\n...\n" + err[-1500:]


def test_rccl_one_rank_bucketed_learner():
    assert os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0") == "0"
    rc, st, err = _child("keep")
    assert st.get("init", {}).get("backend") == "nccl", (rc, st, err)
    assert st["all_reduce"]["ok"], (rc, st, err)
    assert "hooked" in st and st["hooked"]["parts"] == [3], (rc, st, err)  # two bucket cuts + the final part
    assert "plain" in st and st["plain"]["parts"] == [1] and st["plain"]["equal"], (rc, st, err)
    assert rc == 0, (rc, err)


def test_rccl_process_group_teardown_with_graphs_alive():
    """dist.destroy_process_group() while the bucketed learner's captured graphs, its RCCL side
    stream and bucket buffers are all still alive and have just run -- the state DESIGN.md (e)
    once recorded an abort in -- then the graphs released and a normal interpreter exit"""
    rc, st, err = _child("destroy_alive")
    assert "plain" in st and st["plain"]["equal"], (rc, st, err)
    assert "destroyed" in st and "closed" in st, (rc, st, err)
    assert rc == 0, (rc, err)


def test_rccl_bench_shutdown():
    """bench.py's multi-rank exit (reth_amd.dist.shutdown): graphs released, group destroyed,
    normal interpreter exit with rc 0"""
    rc, st, err = _child("shutdown")
    assert "destroyed" in st and st["destroyed"]["initialized"] is False, (rc, st, err)
    assert rc == 0, (rc, err)


def test_rccl_probe_copies_have_no_empty_part():
    """the bench's probe copies of the bucketed learner (cut at the gradient buckets and at the
    probed launches; a probe right before a bucket leaves nothing between the two cuts): no
    empty graph is captured (ApexDQN's _end_part drops such a part) and the result equals the
    unhooked, unprobed loop's"""
    rc, st, err = _child("probe")
    assert "probe" in st, (rc, st, err)
    assert st["probe"]["empty"] == 0 and st["probe"]["equal"], (rc, st, err)
    assert rc == 0, (rc, err)
