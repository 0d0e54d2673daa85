"""Child process of tests/test_apex_gpu.py::test_overlapped_allreduce_stream_edges (run with
GPU_MAX_HW_QUEUES=16 so the loop's streams get hardware queues of their own).  Checks the
data-parallel learner's cross-stream edges in ApexDQN._learner_replay."""
import torch


class _DelayedMarkerReduce:
    """a stream-ordered stand-in for the RCCL all-reduce: on the stream it is
    called on, snapshot the bucket, spin ~10 ms (the side-stream bucket only: a spin on the
    learner stream would delay the final part by itself), then overwrite it with a marker.
    RCCL enqueues asynchronously exactly like this, while the gloo path of GradAllReduce
    host-synchronises -- so only a stand-in like this exposes a missing cross-stream edge."""

    MARK = 1e-3

    def __init__(self):
        self.snaps = []

    def __call__(self, params, grads=None):  # eager learner: nothing to reduce
        pass

    def reduce(self, grads, key="all"):
        self.snaps.append((key, [t.detach().clone() for t in grads]))
        if key == ("bucket", 0):
            torch.cuda._sleep(25_000_000)
        for t in grads:
            t.fill_(self.MARK)


def main():
    """_learner_replay's comm-stream edges: the heads' bucket is reduced on a side stream only
    after the part that computes it (the snapshot never sees the poisoned bucket), and the
    final part (heads split + clip + Adam) consumes the reduced buckets (Adam's exp_avg moves
    towards the marker on every parameter, not towards the local gradients)"""
    from reth_amd.apex import ApexConfig, ApexDQN

    dev = torch.device("cuda:0")
    cfg = ApexConfig(n_actors=16, capacity=1024, batch_size=32, sample_start=64, seed=6, hip_graph=True,
                     dp_hook=True, update_target_interval=1000)
    ax = ApexDQN(cfg, device=dev)
    stand_in = _DelayedMarkerReduce()
    ax.solver.grad_hook = stand_in
    while ax._graphs is None:
        ax.iteration()
    for _ in range(3):  # settle the loop
        ax.iteration()
    G = ax._graphs
    opt, params = ax.solver.optimizer, ax.solver._params
    for _ in range(4):
        torch.cuda.synchronize()
        v = ax._next_learner_variant()
        for kind, item in G["buckets"][v]:
            if kind == "bucket":
                for t in item:
                    t.fill_(float("nan"))
        torch.cuda.synchronize()
        stand_in.snaps.clear()
        before = [opt.state[p]["exp_avg"].clone() for p in params]
        ax.iteration()
        torch.cuda.synchronize()
        assert [k for k, _ in stand_in.snaps] == [("bucket", 0), ("bucket", 1)]
        for _, snap in stand_in.snaps:
            assert all(bool(torch.isfinite(t).all()) for t in snap), "a bucket was reduced before it was computed"
        coef = min(cfg.clip_value / (float(opt.total_norm[0]) + 1e-6), 1.0)
        for p, mb in zip(params, before):
            want = mb + 0.1 * (stand_in.MARK * coef - mb)
            torch.testing.assert_close(opt.state[p]["exp_avg"], want, rtol=1e-5, atol=1e-9)
    ax.close()
    print("stream edges OK")


if __name__ == "__main__":
    main()
