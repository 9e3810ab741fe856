"""Checkpoint I/O in the reference's `latest.pt` layout (train.py:126-130, eval.py:66-112) plus resume.

File = torch.save of a dict with
  * "agent_state_dict": Dreamer.state_dict() — the reference's keys and shapes, including the `_frozen_*` aliases
    (BlockLinear (O/G, I/G, G), conv (Co, Ci, k, k)); eval.py's `agent.load_state_dict(ckpt["agent_state_dict"])`
    works on either implementation's file;
  * "optims_state_dict": {"_optimizer": LaProp state, "_scheduler.optimizer": the same} — the two paths
    tools.recursively_collect_optim_state_dict (utils/tools.py:298-318) finds for the reference agent (the optimizer,
    and again through the LambdaLR's `.optimizer`), in torch.optim.Optimizer.state_dict() form: state index i is
    Dreamer._named_params[i] (the reference's parameter order, dreamer.py:196-206);
  * "resume" (this implementation only; the reference saves once at the end and cannot resume): update counters
    that drive the LR warm-up, the slow-critic schedule and the per-update noise seed, so a resumed run continues
    the same sequence of updates. Everything in the file is tensors / plain Python values: it loads with
    torch.load(..., weights_only=True).
"""
from __future__ import annotations

import os

import torch


def collect_optim_state_dict(agent):
    """tools.recursively_collect_optim_state_dict(agent) for this agent: its one optimizer, reached twice as in the
    reference (agent._optimizer and agent._scheduler.optimizer; one state_dict object, so torch.save stores the
    moments once)."""
    sd = agent._optimizer.state_dict()
    return {"_optimizer": sd, "_scheduler.optimizer": sd}


def checkpoint_items(agent):
    seen, osd = {}, {}  # the same optimizer state under two keys: converted once, stored once
    for k, v in collect_optim_state_dict(agent).items():
        if id(v) not in seen:
            seen[id(v)] = _to_cpu(v)
        osd[k] = seen[id(v)]
    return {
        "agent_state_dict": {k: v.detach().cpu() for k, v in agent.state_dict().items()},
        "optims_state_dict": osd,
        "resume": {"updates": int(agent._updates), "slow_value_updates": int(agent._slow_value_updates),
                   "optimizer_host_steps": int(agent._optimizer.host_steps), "seed_base": int(agent._seed_base),
                   "ema_updates": int(getattr(agent, "_ema_updates", 0)),
                   "moment_layout": "reference"},
    }


def save_checkpoint(agent, path):
    """Write `path` atomically (temp file + rename), so an interrupted save never leaves a torn latest.pt."""
    tmp = f"{path}.tmp"
    torch.save(checkpoint_items(agent), tmp)
    os.replace(tmp, path)
    return path


def load_checkpoint(agent, path, map_location=None):
    """Load a file written by save_checkpoint or by the reference's train.py into `agent` (weights, LaProp moments
    and step, and — when present — the resume counters). Returns the loaded dict."""
    ckpt = torch.load(path, map_location=map_location or "cpu", weights_only=True)
    agent.load_state_dict(ckpt["agent_state_dict"])
    opt = ckpt.get("optims_state_dict", {})
    res = ckpt.get("resume")
    if "_optimizer" in opt:  # the reference's train.py and this module both write reference-layout moments
        ref = not res or res.get("moment_layout") == "reference"
        agent._optimizer.load_state_dict(_to_device(opt["_optimizer"], agent.device),
                                         internal_layout=False if ref else None)
    if res:
        agent._updates = int(res["updates"])
        agent._slow_value_updates = int(res["slow_value_updates"])
        agent._optimizer.host_steps = int(res["optimizer_host_steps"])
        if hasattr(agent, "_ema_updates"):  # DreamerPro's EMA / prototype-freeze counter
            agent._ema_updates = int(res.get("ema_updates", 0))
        agent._seed_base = int(res["seed_base"])
    return ckpt


def _to_cpu(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu()
    if isinstance(x, dict):
        return {k: _to_cpu(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_cpu(v) for v in x)
    return x


def _to_device(x, device):
    if isinstance(x, torch.Tensor):
        return x.to(device)
    if isinstance(x, dict):
        return {k: _to_device(v, device) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_device(v, device) for v in x)
    return x
