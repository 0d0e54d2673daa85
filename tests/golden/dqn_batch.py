"""Seeded learner batches shared by tests/golden/make_golden.py (which runs the reference's
DQNSolver.update on them) and the GPU tests that replay them: the frames are regenerated
from the seed on both sides (numpy's PCG64 stream is platform independent), so the
fixture stores only their SHA-256, not 2 x B x 28,224 random bytes."""
import hashlib

import numpy as np


def apex_batch(seed, B, A):
    """(s0, s1 uint8 [B, 4, 84, 84], a int64, r f32, done f32, isw f64) in the apex learner's
    column dtypes (test/apex-dqn/worker.py:47-51 casts, the sampler's f64 IS weights)"""
    rng = np.random.default_rng(seed)
    s0 = rng.integers(0, 256, (B, 4, 84, 84), dtype=np.uint8)
    s1 = rng.integers(0, 256, (B, 4, 84, 84), dtype=np.uint8)
    a = rng.integers(0, A, B).astype(np.int64)
    r = rng.choice(np.array([-1.0, 0.0, 1.0], np.float32), B).astype(np.float32)
    done = (rng.random(B) < 0.05).astype(np.float32)
    isw = rng.random(B) * 0.8 + 0.2
    return s0, s1, a, r, done, isw


def frames_sha(s0, s1):
    h = hashlib.sha256(np.ascontiguousarray(s0).tobytes())
    h.update(np.ascontiguousarray(s1).tobytes())
    return h.hexdigest()
