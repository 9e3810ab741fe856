"""Helpers to rebuild golden-case inputs for the oracle / product (tests only)."""
import os
import zlib

import numpy as np
import torch

from oracle.init import params_for
from oracle.ref_cpu import Spec
from sdreamer.config import load_config

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

CASES = {
    "proprio_dreamer": ("dmc/proprio", {"position": (3,), "velocity": (2,)}),
    "walker_r2": ("dmc/cnn", {"image": (64, 64, 3)}),
    "walker_r2_nowarm": ("dmc/cnn", {"image": (64, 64, 3)}, ["model.warmup=0"]),
    "walker_infonce": ("dmc/cnn", {"image": (64, 64, 3)}, ["model.rep_loss=infonce"]),
    "walker_r2aug": ("dmc/cnn", {"image": (64, 64, 3)}, ["model.r2dreamer.aug.enabled=True"]),
    "walker_pro": ("dmc/cnn", {"image": (64, 64, 3)}, ["model.rep_loss=dreamerpro"]),
    "walker_dreamer": ("dmc/walker_dreamer", {"image": (64, 64, 3)}),
    "atari_r2": ("dmc/atari_breakout", {"image": (64, 64, 3)}),
    "maze_r2": ("dmc/memory_maze", {"image": (64, 64, 3)}),
}


def case_overrides(name):
    """config overrides of a case beyond its config file (e.g. the rep_loss variant)"""
    return list(CASES[name][2]) if len(CASES[name]) > 2 else []


def load_case(name):
    z = dict(np.load(os.path.join(HERE, name + ".npz")))
    cfg_name, obs = CASES[name][:2]
    H = int(z["meta_H"])
    cfg = load_config(cfg_name, ["device=cpu", "model.compile=False", f"model.imag_horizon={H}"] + case_overrides(name))
    spec = Spec(cfg.model, obs, int(z["meta_A"]), bool(z["meta_discrete"]))
    params = params_for(spec.shapes, int(z["meta_param_seed"]))
    return z, cfg, spec, params, obs


def batch(z, u, obs, device="cpu"):
    data = {}
    for k in list(obs) + ["action", "reward", "is_first", "is_terminal", "is_last"]:
        v = torch.from_numpy(z[f"u{u}_in_{k}"])
        if k in obs and len(obs[k]) == 3:
            v = v.float() / 255.0  # Dreamer.preprocess, dreamer.py:710-713
        data[k] = v.to(device)
    return data


def initial(z, u, spec, device="cpu"):
    idx = torch.from_numpy(z[f"u{u}_in_init_stoch"].astype(np.int64))
    stoch = torch.nn.functional.one_hot(idx, spec.K).float()
    deter = torch.from_numpy(z[f"u{u}_in_init_deter"])
    return stoch.to(device), deter.to(device)


def sample_idx(name, numel, n=32):
    rng = np.random.default_rng([7, zlib.crc32(name.encode())])
    return np.sort(rng.choice(numel, size=min(n, numel), replace=False))
