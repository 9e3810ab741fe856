"""Checkpoint save / resume (sdreamer/checkpoint.py) in the reference's latest.pt layout (train.py:126-130).

A run of 5 updates equals 3 updates -> save -> fresh agent -> load -> 2 updates, bit for bit (weights, LaProp
moments and step, ReturnEMA state, update counters all restored); the file loads with weights_only=True and holds
every reference state_dict key (incl. the _frozen_* aliases) with the reference shapes."""
import os

import pytest
import torch

from golden_io import batch, initial
from test_gpu_dreamer import build_agent

pytestmark = pytest.mark.gpu


def _step(ag, z, spec, obs, u):
    data = batch(z, u % 2, obs, "cuda")
    init = initial(z, u % 2, spec, "cuda")
    _, mets = ag.update_batch(data, init, 900 + u)
    return {k: float(v) for k, v in mets.items() if k.startswith("loss/")}


def test_save_resume_bit_exact(tmp_path):
    from sdreamer.checkpoint import load_checkpoint, save_checkpoint
    a, z, spec, obs = build_agent("walker_r2")
    ref = [_step(a, z, spec, obs, u) for u in range(5)]
    sd_ref = {k: v.detach().clone() for k, v in a.state_dict().items()}
    opt_ref = a._optimizer.state_dict()

    b, _, _, _ = build_agent("walker_r2")
    got = [_step(b, z, spec, obs, u) for u in range(3)]
    path = save_checkpoint(b, os.path.join(tmp_path, "latest.pt"))
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    assert set(ckpt) >= {"agent_state_dict", "optims_state_dict"} and "_optimizer" in ckpt["optims_state_dict"]
    asd = ckpt["agent_state_dict"]
    for k, shape in spec.shapes.items():
        assert k in asd and tuple(asd[k].shape) == tuple(shape), k
    assert any(k.startswith("_frozen_") for k in asd)

    c, _, _, _ = build_agent("walker_r2")  # fresh initial weights, then resume
    load_checkpoint(c, path)
    assert c._updates == 3
    got += [_step(c, z, spec, obs, u) for u in range(3, 5)]
    assert got == ref
    sd = c.state_dict()
    for k, v in sd_ref.items():
        assert torch.equal(sd[k], v), k
    opt = c._optimizer.state_dict()
    assert opt["state"].keys() == opt_ref["state"].keys()
    for i, s in opt_ref["state"].items():
        assert s["step"] == opt["state"][i]["step"]
        assert torch.equal(s["exp_avg"], opt["state"][i]["exp_avg"])
        assert torch.equal(s["exp_avg_sq"], opt["state"][i]["exp_avg_sq"])
