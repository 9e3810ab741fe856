"""sdreamer — MI355X-native (gfx950) Dreamer world-model / imagination training path.

Drop-in surface of the reference's hot path (world_model/{dreamer,rssm,networks}.py, utils/{buffer,optim}.py);
all compute runs in libsdhip.so (HIP/CDNA4 kernels, include/sdhip.h) — importing the model modules without the
library raises (no CPU fallback).
"""
from .config import Config, load_config  # noqa: F401

__all__ = ["Config", "load_config"]
