"""On-device weights broadcast: a latest-wins slot with a version counter.

Replaces the perwez PUB/SUB with CONFLATE used for learner -> actor weights
(perwez/perwez/client/socket.py:302-328; test/apex-dqn/trainer.py:39-41 sends every
`send_weights_interval` updates, worker.py:37-41 loads when more than
`recv_weights_interval` steps passed and a message is waiting).  Learner and actors of a
GPU share its HBM, so publishing is one fused device copy of the parameters into the slot
and acquiring is one copy out of it; conflation falls out of overwriting the slot.
Versions are host integers (the publisher and the consumers run in one process).
The torch.save stream format stays available through DQNSolver.save_weights/load_weights.
"""
import torch


class WeightsSlot:
    def __init__(self, module):
        self._slot = [p.detach().clone() for p in module.parameters()]
        self.version = 0

    @torch.no_grad()
    def publish(self, module):
        torch._foreach_copy_(self._slot, [p.detach() for p in module.parameters()])
        self.version += 1

    @torch.no_grad()
    def acquire(self, module):
        torch._foreach_copy_([p for p in module.parameters()], self._slot)
        if getattr(module, "dueling", False) and hasattr(module, "freeze_heads"):
            module.freeze_heads()  # the actor's cached merged heads follow its parameters
        return self.version


class WeightsSubscriber:
    """the actor side: reload when `interval` actor steps passed and something newer exists"""

    def __init__(self, slot, interval):
        self.slot, self.interval = slot, int(interval)
        self.loaded_version = 0
        self.prev_load = 0

    def maybe_load(self, module, cur_step):
        if cur_step - self.prev_load > self.interval and self.slot.version > self.loaded_version:
            self.loaded_version = self.slot.acquire(module)
            self.prev_load = cur_step
            return True
        return False
