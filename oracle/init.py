"""Deterministic parameter values for parity work (test infrastructure only).

Reference, oracle and product are given IDENTICAL weights by name through this function, so fixtures need
not carry 12M-parameter state dicts. Values are not the reference initialiser (tools.py:76-100); they are
dense, non-zero random values of the right scale so every gradient path is exercised (the reference's
zero-outscale heads, base.yaml:353,414, would zero several paths at init).
"""
import zlib

import numpy as np


def param_value(name: str, shape, seed: int = 0) -> np.ndarray:
    rng = np.random.default_rng([int(seed), zlib.crc32(name.encode())])
    shape = tuple(int(s) for s in shape)
    if name.endswith("last.bias") and shape[0] > 1 and (name.startswith("reward") or "value" in name):
        # symexp two-hot heads (255 bins up to +-4.8e8): keep the mass near the centre bins as a trained
        # head does; random mass on the extreme bins makes TwoHot.mode ill-conditioned (distributions.py:78-98)
        c = (shape[0] - 1) / 2
        return (-0.5 * np.abs(np.arange(shape[0]) - c) + 0.05 * rng.standard_normal(shape)).astype(np.float32)
    if len(shape) == 1:
        if name.endswith("bias"):
            return (0.05 * rng.standard_normal(shape)).astype(np.float32)
        if name.endswith("ema_vals"):
            return np.zeros(shape, np.float32)
        return (1.0 + 0.1 * rng.standard_normal(shape)).astype(np.float32)  # RMSNorm scale
    if len(shape) == 2:
        fan_in = shape[1]
    elif len(shape) == 3:  # BlockLinear (O/G, I/G, G): torch fan_in = I/G * G
        fan_in = shape[1] * shape[2]
    else:  # conv (Co, Ci, kh, kw)
        fan_in = int(np.prod(shape[1:]))
    std = 1.0 / np.sqrt(fan_in)
    if name.endswith("last.weight") and (name.startswith("reward") or "value" in name):
        std *= 0.1
    return (std * rng.standard_normal(shape)).astype(np.float32)


def params_for(shapes: dict, seed: int = 0) -> dict:
    return {k: param_value(k, v, seed) for k, v in shapes.items()}
