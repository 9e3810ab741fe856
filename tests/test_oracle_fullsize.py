"""The CPU oracle against the REAL reference at a BASELINE size (CPU, no GPU): tests/golden/full_<case>.npz holds the
reference's own update() outputs on tests/fullsize_io.py inputs (gen_golden.py `full`). This pins the restatement
beyond the golden sizes (B <= 4, L <= 16): same posterior / imagined indices (near-tie rule), deter and returns at
fp32 tolerance, every loss, the ReturnEMA state and the sampled LaProp moments / parameter steps, for all four
full-size cases (C5's L = 256, deter 4096 update takes minutes on 8 cores). test_gpu_fullsize.py then holds
the product to both the reference fixture and this oracle (teacher-forced) at the same sizes.

The four full-size oracle updates take ~10-25 min of CPU together, so they run only with SDREAMER_ORACLE_FULLSIZE=1
(the default CPU suite must stay within minutes); the last full run's log is profiles/r03_oracle_fullsize.txt."""
import os

import numpy as np
import pytest
import torch

from fullsize_io import FULL, OVERRIDES, PARAM_SEED, SEED, full_inputs, load_fixture, sample_idx
from oracle import noise as nz
from oracle.init import params_for
from oracle.ref_cpu import OracleAgent, Spec, st_gumbel_sample
from parity import assert_close, compare_indices, imag_margins, post_margins, ulp
from sdreamer.config import load_config


def test_fixtures_present():
    for name, (cfg_name, ovr, obs, A, discrete, B, L, H) in FULL.items():
        z = load_fixture(name)
        assert z is not None, name
        assert (int(z["meta_B"]), int(z["meta_L"]), int(z["meta_H"]), int(z["meta_seed"]),
                int(z["meta_param_seed"])) == (B, L, H, SEED, PARAM_SEED), name
        assert z["post_idx"].shape[:2] == (B, L) and z["imag_idx"].shape[1] == H + 1, name
        assert z["imag_ret"].shape == (B * L // int(z["meta_row_stride"]), H), name


def test_teacher_forcing_changes_only_the_hard_sample():
    g = torch.zeros(2, 3, 4)
    lg = torch.randn(2, 3, 4).log_softmax(-1)
    a = st_gumbel_sample(lg, g)
    idx = a.argmax(-1)
    k = (idx[1, 2] + 1) % 4
    b = st_gumbel_sample(lg, g, ((np.array([1]), np.array([2])), np.array([int(k)])))
    assert int(b[1, 2].argmax()) == int(k)
    mask = torch.ones(2, 3, dtype=torch.bool)
    mask[1, 2] = False
    assert torch.equal(a[mask], b[mask])
    soft = lg.softmax(-1)
    assert torch.allclose(b[1, 2] - torch.nn.functional.one_hot(k, 4).float(), -soft[1, 2] + soft[1, 2])


@pytest.mark.skipif(os.environ.get("SDREAMER_ORACLE_FULLSIZE") != "1",
                    reason="minutes of CPU per case: set SDREAMER_ORACLE_FULLSIZE=1 (log: profiles/r03_oracle_fullsize.txt)")
@pytest.mark.parametrize("name", list(FULL))
def test_oracle_matches_reference_fullsize(name):
    cfg_name, ovr, obs, A, discrete, B, L, H = FULL[name]
    cfg = load_config(cfg_name, ["device=cpu"] + ovr + OVERRIDES)
    spec = Spec(cfg.model, obs, A, discrete)
    params = params_for(spec.shapes, PARAM_SEED)
    data_np, init_np = full_inputs(name, spec.K, spec.S, spec.D)
    z = load_fixture(name)
    torch.set_num_threads(8)
    orc = OracleAgent(spec, params)
    data = {k: torch.from_numpy(v) for k, v in data_np.items()}
    data["image"] = data["image"].float() / 255.0
    keep = {}
    (ps, pd), losses, mets = orc.update(data, tuple(torch.from_numpy(v) for v in init_np), SEED, keep=keep)
    plog = keep["post_logit"].detach().numpy()
    dv = compare_indices(ps.argmax(-1).numpy(), z["post_idx"].astype(np.int64),
                         lambda: post_margins(plog, SEED, spec.unimix), "oracle posterior vs reference")
    assert_close(pd.detach().numpy()[..., ::max(1, spec.D // 8)], z["post_deter"], 1e-5, 1e-5, "post_deter",
                 mask=dv[..., None])
    rs = int(z["meta_row_stride"])
    N, SK = B * L, spec.SK
    rows = np.arange(0, N, rs)
    feat = keep["imag_feat"].numpy()[rows]

    def im():
        m = imag_margins(keep["imag_prior_logit"].numpy()[rows], SEED, spec.unimix)
        return np.concatenate([np.full((len(rows), 1, spec.S), np.inf, np.float32), m], 1)

    idv = compare_indices(feat[..., :SK].reshape(len(rows), H + 1, spec.S, spec.K).argmax(-1),
                          z["imag_idx"].astype(np.int64), im, "oracle imagined indices vs reference")
    idv = idv | dv.reshape(-1)[rows][:, None]
    assert_close(feat[..., SK::max(1, spec.D // 4)], z["imag_deter"], 1e-5, 1e-5, "imag_deter", mask=idv[..., None])
    ok = ~idv.any(1)
    assert_close(keep["ret"].numpy()[rows, :, 0], z["imag_ret"], 1e-4, 1e-4, "imag_ret", mask=~ok[:, None])
    flip = bool(idv.any())
    for k, v in losses.items():
        ref = float(z[f"m_loss/{k}"])
        tol = 1e-5 if not flip else 1e-2
        assert abs(float(v.detach()) - ref) <= tol * abs(ref) + 1e-6, (k, float(v.detach()), ref)
    if not flip:
        assert_close(orc.ema_vals.numpy(), z["ema_vals"], 1e-5, 1e-6, "ema_vals")
        assert_close(keep["rret"].detach().numpy()[..., 0], z["replay_ret"], 1e-4, 1e-4, "replay_ret")
    for k in spec.shapes:
        idx = sample_idx(k, int(np.prod(spec.shapes[k])))
        st = orc.state[id(orc.P[k])]
        vmax = float(z[f"v_{k}__max"])
        v = st["exp_avg_sq"].reshape(-1).numpy()
        assert_close(v[idx], z[f"v_{k}__s"], 1e-3, 1e-5 * vmax + 1e-30, f"exp_avg_sq {k}")
        p1 = orc.P[k].detach().reshape(-1).numpy()
        tiny = np.sqrt(np.maximum(z[f"v_{k}__s"], 0)) < 1e-3 * np.sqrt(vmax)
        assert_close(p1[idx], z[f"p_{k}__s"], 0, 4 * ulp(z[f"p_{k}__s"]) + 1e-3 * 4e-5, f"param {k}", mask=tiny)
