"""The reference's reth/examples/dqn/run.py on this build: CartPole DQN, the in-process
prioritized buffer in HBM, the learner update through the HIP TD/Huber + clip/Adam path.

    python examples/cartpole_dqn.py [max_ts]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from reth_amd.buffer import PrioritizedBuffer  # noqa: E402
from reth_amd.presets import get_replay_buffer, get_solver, get_trainer, get_worker  # noqa: E402

BATCH_SIZE = 64
MAX_TS = 100000


def main(max_ts=MAX_TS, config=os.path.join(os.path.dirname(os.path.abspath(__file__)), "cartpole_dqn.yaml")):
    solver = get_solver(config)
    worker = get_worker(config, solver=solver)  # shared solver
    trainer = get_trainer(config, solver=solver)
    buffer = get_replay_buffer(config)
    assert isinstance(buffer, PrioritizedBuffer)
    buffer.append_batch(worker.step_batch(1000))  # init buffer
    for _ in range(max_ts):
        data = worker.step_batch(BATCH_SIZE)  # worker
        solver.calc_loss(data)
        buffer.append_batch(data)
        data, indices, weights = buffer.sample(BATCH_SIZE)  # trainer
        loss = trainer.step(data)
        buffer.update_priorities(indices, loss)
    return worker, trainer, buffer


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else MAX_TS)
