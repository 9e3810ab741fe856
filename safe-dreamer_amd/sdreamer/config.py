"""Hydra-compatible configuration surface for the Dreamer hot path.

Mirrors the key layout of configs/base.yaml + configs/dmc/*.yaml in the reference
(configs/base.yaml:13-432, composed through `defaults: [/base@_global_, _self_]`, configs/dmc/cnn.yaml:9-11).
hydra/omegaconf are not installed in this image, so this module provides:
  * `load_config(name, overrides)` — composes a YAML config with its `defaults` list,
    resolves `${a.b.c}` interpolations and applies Hydra-style `key=value` CLI overrides;
  * `Config` — an attribute dict that supports attribute assignment (the reference mutates
    `config.actor.shape/dist`, world_model/dreamer.py:73-82) and `dict(cfg.loss_scales)` (dreamer.py:94).
If OmegaConf objects are passed in instead (real Hydra), every consumer in this package only uses
attribute/item access, so both work.
"""
from __future__ import annotations

import copy
import os
import re

import yaml

class _Loader(yaml.SafeLoader):
    """SafeLoader that, like OmegaConf, reads '4e-5' / '5e5' as floats (YAML 1.1 wants a dot)."""


_Loader.add_implicit_resolver(
    "tag:yaml.org,2002:float",
    re.compile(r"""^(?:[-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
                  |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
                  |\.[0-9_]+(?:[eE][-+][0-9]+)?
                  |[-+]?\.(?:inf|Inf|INF)
                  |\.(?:nan|NaN|NAN))$""", re.X),
    list("-+0123456789."),
)

_CFG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "configs")
_INTERP = re.compile(r"\$\{([^}]+)\}")


class Config(dict):
    """dict with attribute access; nested dicts become Config on construction."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        for k, v in list(self.items()):
            self[k] = _wrap(v)

    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError as e:
            raise AttributeError(name) from e

    def __setattr__(self, name, value):
        self[name] = _wrap(value)

    def __delattr__(self, name):
        del self[name]

    def __deepcopy__(self, memo):
        return Config({k: copy.deepcopy(v, memo) for k, v in self.items()})

    def to_dict(self):
        return {k: (v.to_dict() if isinstance(v, Config) else v) for k, v in self.items()}


def _wrap(v):
    if isinstance(v, Config):
        return v
    if isinstance(v, dict):
        return Config(v)
    if isinstance(v, list):
        return [_wrap(x) for x in v]
    return v


def _deep_merge(dst: dict, src: dict) -> dict:
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _deep_merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


def _load_yaml(name: str, cfg_dir: str) -> dict:
    path = name if (os.path.isabs(name) and os.path.exists(name + ("" if name.endswith(".yaml") else ".yaml"))) \
        else os.path.join(cfg_dir, name.lstrip("/"))
    if not path.endswith(".yaml"):
        path += ".yaml"
    with open(path) as f:
        raw = yaml.load(f, Loader=_Loader) or {}
    defaults = raw.pop("defaults", None)
    if not defaults:
        return raw
    out: dict = {}
    for d in defaults:
        if d == "_self_":
            _deep_merge(out, raw)
            continue
        sub = d if isinstance(d, str) else next(iter(d.values()))
        sub = sub.split("@")[0]  # "/base@_global_" → package _global_ (merged at root)
        _deep_merge(out, _load_yaml(sub, cfg_dir))
    if "_self_" not in defaults:
        _deep_merge(out, raw)
    return out


def _lookup(root: dict, dotted: str):
    cur = root
    for part in dotted.split("."):
        cur = cur[part]
    return cur


def _resolve(node, root, depth=0):
    if depth > 32:
        raise ValueError("interpolation cycle")
    if isinstance(node, dict):
        for k in list(node):
            node[k] = _resolve(node[k], root, depth)
        return node
    if isinstance(node, list):
        return [_resolve(x, root, depth) for x in node]
    if isinstance(node, str):
        m = _INTERP.fullmatch(node.strip())
        if m:  # whole-value interpolation keeps the referenced type
            return _resolve(copy.deepcopy(_lookup(root, m.group(1))), root, depth + 1)
        if _INTERP.search(node):
            return _INTERP.sub(lambda mm: str(_resolve(copy.deepcopy(_lookup(root, mm.group(1))), root, depth + 1)), node)
    return node


def _parse_value(text: str):
    return yaml.load(text, Loader=_Loader) if text != "" else ""


def apply_overrides(raw: dict, overrides) -> dict:
    for ov in overrides or ():
        key, _, val = ov.lstrip("+").partition("=")
        cur = raw
        parts = key.split(".")
        for p in parts[:-1]:
            cur = cur.setdefault(p, {})
        cur[parts[-1]] = _parse_value(val)
    return raw


def load_config(name: str = "dmc/cnn", overrides=None, cfg_dir: str | None = None) -> Config:
    """Compose `name` (relative to the config dir), apply `k=v` overrides, resolve `${}`."""
    raw = _load_yaml(name, cfg_dir or _CFG_DIR)
    raw = apply_overrides(raw, overrides)
    raw = _resolve(raw, raw)
    return Config(raw)


def as_float(x):
    """YAML 1.1 reads '5e5' / '1e4' as strings; the reference casts with float()/int()."""
    return float(x)
