"""Full-size parity cases (BASELINE.json configs at their real sizes) and their deterministic inputs.

Shared by tests/golden/gen_golden.py (which runs the REAL reference's update() on these inputs in the build
container and stores a compact fixture, tests/golden/full_<case>.npz), tests/test_gpu_fullsize.py (product vs the
teacher-forced oracle AND vs that fixture) and bench.py's parity leg (WM-loss delta at the headline size).
Test infrastructure: the inputs are regenerated from a seed, so the fixtures carry only outputs.
"""
import os
import zlib

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
IMG = {"image": (64, 64, 3)}
FULL = {  # name: (config, overrides, obs, act_dim, discrete, B, L, H)
    "C2_walker_r2": ("dmc/cnn", [], IMG, 6, False, 16, 64, 15),
    "C3_walker_dreamer_shard": ("dmc/walker_dreamer", ["batch_size=8"], IMG, 6, False, 8, 64, 15),
    "C4_atari": ("dmc/atari_breakout", [], IMG, 4, True, 32, 64, 15),
    "C5_maze": ("dmc/memory_maze", [], IMG, 6, True, 16, 256, 25),
}
SEED = 4242  # noise seed of the one update (oracle/noise.py streams)
PARAM_SEED = 0  # oracle/init.py params_for seed
# every case runs with model.warmup=0: the first LaProp step is lr = 4e-5 per element, so parameter steps resolve
OVERRIDES = ["model.compile=False", "model.warmup=0"]
# imagined rows stored in the fixture: every ROW_STRIDE-th start row (keeps each fixture well under 1 MB)
ROW_STRIDE = {"C2_walker_r2": 2, "C3_walker_dreamer_shard": 1, "C4_atari": 4, "C5_maze": 8}


def full_inputs(name, K, S, D):
    """The case's replay batch (uint8 images, actions, rewards, episode flags) and initial latents."""
    _, _, obs, A, discrete, B, L, _ = FULL[name]
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    d = {"image": rng.integers(0, 256, size=(B, L, 64, 64, 3), dtype=np.uint8)}
    if discrete:
        d["action"] = np.eye(A, dtype=np.float32)[rng.integers(0, A, size=(B, L))]
    else:
        d["action"] = rng.uniform(-1, 1, size=(B, L, A)).astype(np.float32)
    d["reward"] = rng.uniform(0, 1, size=(B, L, 1)).astype(np.float32)
    first = rng.random((B, L, 1)) < 0.02
    first[:, 0] = True
    d["is_first"] = first
    term = rng.random((B, L, 1)) < 0.02
    d["is_terminal"] = term
    d["is_last"] = term | (rng.random((B, L, 1)) < 0.01)
    idx = rng.integers(0, K, size=(B, S))
    init = (np.eye(K, dtype=np.float32)[idx], (0.5 * rng.standard_normal((B, D))).astype(np.float32))
    return d, init


def fixture_path(name):
    return os.path.join(HERE, f"full_{name}.npz")


def load_fixture(name):
    p = fixture_path(name)
    return dict(np.load(p)) if os.path.exists(p) else None


def sample_idx(name, numel, n=32):
    """The parameter elements a fixture samples (same rule as the golden cases)."""
    rng = np.random.default_rng([7, zlib.crc32(name.encode())])
    return np.sort(rng.choice(numel, size=min(n, numel), replace=False))
