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


@pytest.mark.parametrize("name", ["walker_r2", "walker_dreamer", "proprio_dreamer", "atari_r2", "maze_r2", "walker_pro"])
def test_optim_state_layout_matches_reference(name, tmp_path):
    """optims_state_dict as the reference's train.py:126-130 writes it (tools.recursively_collect_optim_state_dict,
    tools.py:298-318; golden tests/golden/optim_layout.json recorded from the reference after its two updates): the
    same keys ("_optimizer", "_scheduler.optimizer"), state_dict structure and param_group values, and LaProp state
    index i <-> Dreamer._named_params[i] in the reference's order (dreamer.py:196-206; the moments of index i are
    checked element-wise against the reference's by test_update_matches_reference). Round-trips through the file."""
    import json
    from golden_io import HERE
    from sdreamer.checkpoint import load_checkpoint, save_checkpoint
    lay = json.load(open(os.path.join(HERE, "optim_layout.json")))[name]
    ag, z, spec, obs = build_agent(name)
    assert list(ag._named_params) == lay["named_params"]
    sd_name = {id(p): n for n, p in ag.named_parameters()}  # state_dict key of each _named_params entry
    shape_of = {n: spec.shapes[sd_name[id(p)]] for n, p in ag._named_params.items()}
    for u in range(2):
        ag.update_batch(batch(z, u, obs, "cuda"), initial(z, u, spec, "cuda"), int(z[f"u{u}_seed"]))
    path = save_checkpoint(ag, os.path.join(tmp_path, "latest.pt"))
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    osd = ckpt["optims_state_dict"]
    assert list(osd) == lay["optims_keys"]
    for key, ref in lay["optimizers"].items():
        sd = osd[key]
        assert sorted(sd) == ref["top_keys"]
        assert len(sd["param_groups"]) == ref["n_groups"]
        g = sd["param_groups"][0]
        assert list(g["params"]) == ref["params"]
        for k, v in ref["group"].items():
            got = list(g[k]) if isinstance(g[k], tuple) else g[k]
            if isinstance(v, float):
                assert abs(got - v) <= 1e-12 * abs(v), (k, got, v)
            else:
                assert got == v, (k, got, v)
        assert len(sd["state"]) == ref["n_state"]
        for i, st in sd["state"].items():
            assert sorted(st) == ref["state_keys"], i
            assert tuple(st["exp_avg"].shape) == tuple(shape_of[lay["named_params"][i]])
    b, _, _, _ = build_agent(name)
    load_checkpoint(b, path)
    o1, o2 = ag._optimizer.state_dict(), b._optimizer.state_dict()
    for i, st in o1["state"].items():
        assert torch.equal(st["exp_avg"], o2["state"][i]["exp_avg"]) and st["step"] == o2["state"][i]["step"]


def test_optim_load_layouts():
    """LaProp.load_state_dict: reference-layout moments (train.py's files and save_checkpoint's) load; internal-layout
    moments of an older file (no `moment_layout` marker) are recognised by shape; a moment whose shape matches
    neither layout raises instead of broadcasting."""
    a, z, spec, obs = build_agent("walker_r2")
    _step(a, z, spec, obs, 0)
    sd = a._optimizer.state_dict()
    arena = a._optimizer.arena
    internal = {"param_groups": sd["param_groups"], "state": {}}
    packed = 0
    for i, st in sd["state"].items():
        lay = a._optimizer.ref_layouts[i]
        conv = (lambda t: t) if lay is None else lay[1]
        packed += lay is not None
        internal["state"][i] = dict(st, exp_avg=conv(st["exp_avg"]).contiguous(),
                                    exp_avg_sq=conv(st["exp_avg_sq"]).contiguous())
    assert packed > 0
    for src in (sd, internal):
        b, _, _, _ = build_agent("walker_r2")
        b._optimizer.load_state_dict(src)
        o = b._optimizer.state_dict()
        for i, st in sd["state"].items():
            assert torch.equal(st["exp_avg"], o["state"][i]["exp_avg"]), i
            assert torch.equal(st["exp_avg_sq"], o["state"][i]["exp_avg_sq"]), i
    b, _, _, _ = build_agent("walker_r2")
    with pytest.raises(ValueError):  # a file that declares reference-layout moments but holds internal ones
        b._optimizer.load_state_dict(internal, internal_layout=False)
    bad = {"param_groups": sd["param_groups"],
           "state": {0: dict(sd["state"][0], exp_avg=torch.zeros(3), exp_avg_sq=torch.zeros(3))}}
    with pytest.raises(ValueError):
        b._optimizer.load_state_dict(bad)
