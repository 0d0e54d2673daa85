"""BASELINE configs[0] on this build: the reference's CartPole DQN loop (reth/examples/dqn/
run.py: Worker -> buffer -> Trainer from one YAML) on the host -- CPU torch solver and a
uniform numpy replay, no GPU.  The GPU path of the same loop is examples/cartpole_dqn.py.

    python examples/cartpole_cpu.py [max_ts]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from reth_amd.presets import get_replay_buffer, get_solver, get_trainer, get_worker  # noqa: E402

BATCH_SIZE = 64
MAX_TS = 100000


def main(max_ts=MAX_TS, config=os.path.join(os.path.dirname(os.path.abspath(__file__)), "cartpole_cpu.yaml")):
    solver = get_solver(config)
    worker = get_worker(config, solver=solver)
    trainer = get_trainer(config, solver=solver)
    buffer = get_replay_buffer(config, device="cpu")
    buffer.append_batch(worker.step_batch(1000))
    for _ in range(max_ts):
        buffer.append_batch(worker.step_batch(1))  # one env step ...
        data = buffer.sample(BATCH_SIZE)            # ... and one update per step (run.py:22-30)
        trainer.step(data)
    return worker, trainer, buffer


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else MAX_TS)
