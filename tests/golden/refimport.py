"""Import the read-only reference (/root/reference) in THIS container, for golden-vector generation only.

Test infrastructure, never shipped and never run on the GPU box (the reference does not exist there).
Recipe from SURVEY.md §8(c): stub the I/O-only modules the hot path never uses for arithmetic
(tensorboard SummaryWriter imported at utils/tools.py:12, tensordict.TensorDict imported at
world_model/dreamer.py:7), pre-register `utils` / `world_model` packages so their __init__ files
(which pull torchrl / multimodal CLIP) are skipped, then import the modules of the path.
"""
import sys
import types

REF = "/root/reference"


def import_reference():
    sys.dont_write_bytecode = True
    if REF not in sys.path:
        sys.path.insert(0, REF)
    # tensorboard stub
    tb = types.ModuleType("torch.utils.tensorboard")

    class SummaryWriter:  # noqa: D401 - stub
        def __init__(self, *a, **k):
            pass

    tb.SummaryWriter = SummaryWriter
    sys.modules["torch.utils.tensorboard"] = tb
    # tensordict stub: only `.shape` is read on the _cal_grad path (dreamer.py:467)
    td = types.ModuleType("tensordict")

    class TensorDict(dict):
        def __init__(self, d=None, batch_size=None, **k):
            super().__init__(d or {})
            self.batch_size = batch_size

        @property
        def shape(self):
            return self.batch_size

    td.TensorDict = TensorDict
    sys.modules["tensordict"] = td
    for pkg in ("utils", "world_model", "world_model.multimodal_encoder", "ablations"):
        m = types.ModuleType(pkg)
        m.__path__ = [REF + "/" + pkg.replace(".", "/")]
        sys.modules[pkg] = m
    mm = sys.modules["world_model.multimodal_encoder"]
    mm.MultimodalEncoder = type("MultimodalEncoder", (), {})
    mm.MultimodalEncoderConfig = type("MultimodalEncoderConfig", (), {})
    ab = types.ModuleType("ablations.ablation_encoders")
    ab.GateOnlyEncoder = type("GateOnlyEncoder", (), {})
    sys.modules["ablations.ablation_encoders"] = ab
    import importlib

    mods = {}
    for name in ("utils.tools", "utils.optim", "world_model.distributions", "world_model.networks",
                 "world_model.rssm", "world_model.dreamer"):
        mods[name] = importlib.import_module(name)
    return mods, TensorDict
