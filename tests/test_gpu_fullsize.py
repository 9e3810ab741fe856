"""Full-size parity: one product update at the BASELINE configs vs (1) the REAL reference's own update() on the same
inputs (tests/golden/full_<case>.npz, written by tests/golden/gen_golden.py `full` in the build container) and (2)
the CPU oracle, teacher-forced at near-tie flips.

The golden cases (test_gpu_dreamer.py) pin the product to the reference at small sizes (B2-4, L4-16); this file runs
it at the sizes the bench runs — the 8192-workgroup encoder grids, 1,024-4,096-row imagination tiles and the
L = 256 BPTT of the deter-4096 model — on identical weights (oracle/init.py params_for), batch, initial latents and
Philox noise (tests/fullsize_io.py):
  C2  walker r2dreamer       B16 L64  H15, 6 continuous actions            (BASELINE configs[1], the bench workload)
  C3  walker dreamer decoder B8  L64  H15 = one rank's shard of B64 on 8 GPUs (configs[2])
  C4  atari-like discrete    B32 L64  H15, 32x32 stoch, 4 one-hot actions  (configs[3])
  C5  memory-maze-like       B16 L256 H25, deter 4096, 6 one-hot actions   (configs[4])

Index rule (BASELINE.json north_star): posterior / imagined latent indices and one-hot actions bit-exact except at
near-ties (top-2 perturbed-logit margin < 1e-5).

Oracle leg, teacher-forced: when the product's sample at a near-tie differs from the oracle's, the oracle is rerun
with the product's index forced at that site (oracle/ref_cpu.py st_gumbel_sample `force`: the hard sample only,
the soft straight-through part untouched), until the two trajectories agree everywhere. Every comparison is then
strict, with no flipped rows to mask: deter / logits 1e-4, imagined returns 1e-3, world-model losses 1e-4
relative, other losses 5e-3, and the FULL tensors of the LaProp second moment (2e-2 rel + 2e-4 of the tensor max)
and of the parameter step (model.warmup=0, lr = 4e-5 per element: 2e-2 rel + 2e-3 of the max step).

Reference leg: the fixture holds the reference's metrics, posterior indices and deter columns, replay returns,
ReturnEMA state, the imagined indices / deter columns / actions / returns of every ROW_STRIDE-th start row, and per
parameter the step and second-moment norms plus 32 sampled elements. The reference cannot be teacher-forced after
the fact, so rows that flipped at a near-tie against it are compared up to the flip; its tolerances are the oracle
leg's while no row flipped against the reference, and only then widen (world-model losses 1e-3, actor-critic
losses 5e-2, sampled moments / steps 5 % of the tensor max) — the report says which applied.

Each case's report (flips forced, errors, times) is printed, and written to $SDREAMER_FULLSIZE_REPORT/<case>.json when set.
"""
import copy
import json
import os
import time

import numpy as np
import pytest
import torch

from fullsize_io import FULL, OVERRIDES, PARAM_SEED, SEED, full_inputs, load_fixture, sample_idx
from oracle import noise as nz
from oracle.init import params_for
from oracle.ref_cpu import OracleAgent, Spec
from parity import MARGIN, assert_close, compare_indices, imag_margins, perturbed_margin, post_margins, ulp
from sdreamer.config import load_config
from test_gpu_dreamer import WM_KEYS, _Spaces, _Sp

pytestmark = pytest.mark.gpu
REPORT_DIR = os.environ.get("SDREAMER_FULLSIZE_REPORT")  # opt-in: the directory for the per-case JSON reports


def _run_product(name, spec, params, data_np, init_np):
    from sdreamer.dreamer import Dreamer
    cfg_name, ovr, obs, A, discrete, B, L, H = FULL[name]
    gcfg = load_config(cfg_name, ["device=cuda:0"] + ovr + OVERRIDES)
    act = _Sp((A,))
    if discrete:
        act.discrete = True
    ag = Dreamer(copy.deepcopy(gcfg.model), _Spaces({k: _Sp(v) for k, v in obs.items()}), act)
    sd = {k: torch.from_numpy(v) for k, v in params.items()}
    for k, sk in spec.slow_names.items():
        sd[sk] = torch.from_numpy(params[k])
    sd["return_ema.ema_vals"] = torch.zeros(2)
    ag.load_state_dict(sd, strict=False)
    data = {k: torch.from_numpy(v).cuda() for k, v in data_np.items()}
    init = tuple(torch.from_numpy(v).cuda() for v in init_np)
    t0 = time.time()
    (ps, pd), mets = ag.update_batch(data, init, SEED)
    torch.cuda.synchronize()
    return ag, ps, pd, mets, time.time() - t0


def _run_oracle(spec, params, data_np, init_np, force):
    orc = OracleAgent(spec, params)
    orc.model.force = force
    cdata = {k: torch.from_numpy(v) for k, v in data_np.items()}
    cdata["image"] = cdata["image"].float() / 255.0
    keep = {}
    (ops_, opd), losses, omets = orc.update(cdata, tuple(torch.from_numpy(v) for v in init_np), SEED, keep=keep)
    return orc, ops_, opd, losses, omets, keep


def _add(force, key, site, k):
    """append (site, index) to the teacher-forcing table entry `key`"""
    if key in force:
        (old_site, old_k) = force[key]
        site = tuple(np.concatenate([a, b]) for a, b in zip(old_site, site))
        k = np.concatenate([old_k, k])
    force[key] = (site, k)


def _next_forcing(spec, seed, p_post, p_imag, p_act, ops_, keep, force):
    """Compare the product's samples with one oracle run; for every row whose first mismatch is a near-tie, force the
    product's index there (posterior flips first: they move every later imagination start row). Returns the number
    of sites forced; asserts that every mismatch it meets is a near-tie."""
    S, Kd = spec.S, spec.K
    o_post = ops_.argmax(-1).numpy()
    neq = p_post != o_post  # (B, L, S)
    if neq.any():
        m = post_margins(keep["post_logit"].detach().numpy(), seed, spec.unimix)
        n = 0
        step_bad = neq.any(-1)
        for b in np.nonzero(step_bad.any(1))[0]:
            t = int(np.argmax(step_bad[b]))
            s = np.nonzero(neq[b, t])[0]
            worst = float(m[b, t, s].max())
            assert worst < MARGIN, f"posterior flip at row {b} step {t} latents {s.tolist()}: margin {worst:.3g}"
            _add(force, ("obs", nz.STREAM_OBS, t), (np.full(len(s), b), s), p_post[b, t, s])
            n += len(s)
        return n
    rfeat = keep["imag_feat"].numpy()
    N, H1 = rfeat.shape[:2]
    o_imag = rfeat[..., :spec.SK].reshape(N, H1, S, Kd).argmax(-1)
    ineq = (p_imag != o_imag).any(-1)  # (N, H1): feat t's latents (img_step t - 1)
    aneq = np.zeros_like(ineq)
    if spec.discrete:
        aneq = p_act != keep["imag_action"].numpy().argmax(-1)
    if not (ineq.any() or aneq.any()):
        return 0
    mi = imag_margins(keep["imag_prior_logit"].numpy(), seed, spec.unimix)  # (N, H, S) of img_step t
    n = 0
    for r in np.nonzero((ineq | aneq).any(1))[0]:
        # the events of a row in time order: feat t's latents (from img_step t - 1) come before the actor sample at t
        ti = int(np.argmax(ineq[r])) if ineq[r].any() else H1
        ta = int(np.argmax(aneq[r])) if aneq[r].any() else H1
        if ti <= ta:
            s = np.nonzero(p_imag[r, ti] != o_imag[r, ti])[0]
            worst = float(mi[r, ti - 1, s].max())
            assert worst < MARGIN, f"imagined flip at row {r} step {ti} latents {s.tolist()}: margin {worst:.3g}"
            _add(force, ("img", nz.STREAM_IMG, ti - 1), (np.full(len(s), r), s), p_imag[r, ti, s])
            n += len(s)
        else:
            lg = keep["imag_actor_logit"][r:r + 1, ta].numpy()
            g = nz.gumbel_block(seed, nz.STREAM_ACT, ta, N, 0, spec.A)[r:r + 1]
            worst = float(perturbed_margin(lg, g, float(spec.actor_dist.unimix_ratio))[0])
            assert worst < MARGIN, f"imagined action flip at row {r} step {ta}: margin {worst:.3g}"
            _add(force, ("act", nz.STREAM_ACT, ta), (np.array([r]),), np.array([p_act[r, ta]]))
            n += 1
    return n


def _loss_tol(k, wm_flip, ac_flip):
    if k in WM_KEYS:
        return 1e-3 if wm_flip else 1e-4
    return 5e-2 if ac_flip else 5e-3


@pytest.mark.parametrize("name", list(FULL))
def test_fullsize_update_matches_reference_and_oracle(name):
    cfg_name, ovr, obs, A, discrete, B, L, H = FULL[name]
    ccfg = load_config(cfg_name, ["device=cpu"] + ovr + OVERRIDES)
    assert int(ccfg.batch_size) == B and int(ccfg.batch_length) == L and int(ccfg.model.imag_horizon) == H
    spec = Spec(ccfg.model, obs, A, discrete)
    params = params_for(spec.shapes, PARAM_SEED)
    data_np, init_np = full_inputs(name, spec.K, spec.S, spec.D)
    S, Kd, SK, N, H1 = spec.S, spec.K, spec.SK, B * L, H + 1
    # ---- product (HIP)
    ag, ps, pd, mets, t_gpu = _run_product(name, spec, params, data_np, init_np)
    p_post = ps.argmax(-1).cpu().numpy()
    ifeat = ag._last["imag_feat_tm"].detach().transpose(0, 1).cpu().numpy()  # (N, H1, F)
    assert ifeat.shape[:2] == (N, H1)
    p_imag = ifeat[..., :SK].reshape(N, H1, S, Kd).argmax(-1)
    iact = ag._last["imag_action_tm"].detach().transpose(0, 1).cpu().numpy()
    p_act = iact.argmax(-1) if discrete else None
    p_ret = ag._last["ret"].detach().cpu().numpy()
    report = {"case": name, "t_gpu_s": round(t_gpu, 2)}
    # ---- oracle (CPU), teacher-forced at near-ties until the trajectories agree
    torch.set_num_threads(16)
    force, forced, runs, t_cpu = {}, 0, 0, 0.0
    while True:
        t0 = time.time()
        orc, ops_, opd, losses, omets, keep = _run_oracle(spec, params, data_np, init_np, force)
        t_cpu += time.time() - t0
        runs += 1
        n = _next_forcing(spec, SEED, p_post, p_imag, p_act, ops_, keep, force)
        if n == 0:
            break
        forced += n
        assert runs <= 6, f"teacher forcing did not converge after {runs} oracle runs ({forced} sites)"
    report.update(oracle_runs=runs, forced_sites=forced, forced_keys=sorted(f"{k[0]}{k[2]}" for k in force),
                  t_cpu_s=round(t_cpu, 2))
    # posterior (rssm.py:140-178): indices now identical everywhere
    assert np.array_equal(p_post, ops_.argmax(-1).numpy())
    ref_logit = keep["post_logit"].detach().numpy()
    assert_close(pd.detach().cpu().numpy(), opd.detach().numpy(), 1e-4, 1e-4, "post_deter")
    assert_close(ag._last["post_logit"].detach().cpu().numpy(), ref_logit, 1e-4, 1e-4, "post_logit")
    prl = ag._last["prior_logit"].detach().cpu().numpy().reshape(ref_logit.shape)
    assert_close(prl, keep["prior_logit"].detach().numpy(), 1e-4, 1e-4, "prior_logit")
    report["oracle_post_deter_maxerr"] = float(np.abs(pd.detach().cpu().numpy() - opd.detach().numpy()).max())
    # imagination (dreamer.py:673-692)
    rfeat = keep["imag_feat"].numpy()
    assert np.array_equal(p_imag, rfeat[..., :SK].reshape(N, H1, S, Kd).argmax(-1))
    assert_close(ifeat[..., SK:], rfeat[..., SK:], 1e-4, 1e-4, "imag_deter")
    assert_close(iact, keep["imag_action"].numpy(), 1e-4, 1e-4, "imag_action")
    assert_close(p_ret, keep["ret"].numpy()[..., 0], 1e-3, 1e-3, "imag_ret")
    report["oracle_imag_deter_maxerr"] = float(np.abs(ifeat[..., SK:] - rfeat[..., SK:]).max())
    # losses (dreamer.py:453-671)
    bad = []
    for k, v in losses.items():
        got, ref = float(mets[f"loss/{k}"]), float(v)
        rel = abs(got - ref) / max(abs(ref), 1e-6)
        report[f"oracle_rel_{k}"] = rel
        if rel > _loss_tol(k, False, False) and abs(got - ref) > 1e-5:
            bad.append((k, got, ref, rel))
    assert not bad, (bad, report)
    # optimizer step (agc.py:15-53, laprop.py:85-116): full second-moment and parameter-step tensors
    ost = ag._optimizer.state_dict()["state"]
    sd_name = {id(p): n for n, p in ag.named_parameters()}
    psd = ag.state_dict()
    got_v, got_dp = {}, {}
    worst_v = 0.0
    for i, prm in enumerate(ag._named_params.values()):
        k = sd_name[id(prm)]
        st = orc.state[id(orc.P[k])]
        v_ref = st["exp_avg_sq"].reshape(-1).numpy().astype(np.float64)
        v = ost[i]["exp_avg_sq"].reshape(-1).cpu().numpy().astype(np.float64)
        vmax = np.abs(v_ref).max()
        assert_close(v, v_ref, 2e-2, 2e-4 * vmax + 1e-30, f"exp_avg_sq {k}")
        worst_v = max(worst_v, float((np.abs(v - v_ref) / (np.abs(v_ref) + 1e-3 * vmax + 1e-30)).max()))
        # LaProp's first step is lr * sign(g): elements whose |g| is within the fp32-vs-split-bf16 rounding of the
        # tensor's gradients (< 1 % of its largest |g|) may flip sign
        tiny = np.sqrt(v_ref) < 1e-2 * np.sqrt(vmax)
        p0 = params[k].reshape(-1).astype(np.float64)
        p_ref = orc.P[k].detach().reshape(-1).numpy()
        d_got = psd[k].detach().reshape(-1).cpu().numpy().astype(np.float64) - p0
        d_ref = p_ref.astype(np.float64) - p0
        assert_close(d_got, d_ref, 2e-2, 2e-3 * np.abs(d_ref).max() + 4 * ulp(p_ref), f"parameter step {k}", mask=tiny)
        got_v[k], got_dp[k] = v, d_got
    report["oracle_worst_v_rel"] = worst_v
    # ---- the reference's own update() at this size (fixture)
    z = load_fixture(name)
    assert z is not None, f"missing tests/golden/full_{name}.npz (python tests/golden/gen_golden.py full {name})"
    assert (int(z["meta_B"]), int(z["meta_L"]), int(z["meta_H"]), int(z["meta_seed"])) == (B, L, H, SEED)
    rs = int(z["meta_row_stride"])
    # posterior indices: margins at the teacher-forced oracle's logits, which equal the reference's up to each row's
    # first flip against the reference (before it both follow the same trajectory)
    dv = compare_indices(p_post, z["post_idx"].astype(np.int64),
                         lambda: post_margins(ref_logit, SEED, spec.unimix), "posterior indices vs reference")
    report["ref_post_rows_flipped"] = int(dv.any(1).sum())
    dcol = max(1, spec.D // 8)
    assert_close(pd.detach().cpu().numpy()[..., ::dcol], z["post_deter"], 1e-4, 1e-4, "post_deter vs reference",
                 mask=dv[..., None])
    rows = np.arange(0, N, rs)
    sub_imag = p_imag[rows]

    def imargin():
        m = imag_margins(keep["imag_prior_logit"].numpy()[rows], SEED, spec.unimix)
        return np.concatenate([np.full((len(rows), 1, S), np.inf, np.float32), m], 1)

    idv = compare_indices(sub_imag, z["imag_idx"].astype(np.int64), imargin, "imagined indices vs reference")
    idv = idv | dv.reshape(-1)[rows][:, None]
    if discrete:
        def amargin():  # the actor samples' perturbed-logit margins (dreamer.py:684; oracle actor_sample)
            lg = keep["imag_actor_logit"].numpy()[rows]
            g = np.stack([nz.gumbel_block(SEED, nz.STREAM_ACT, t, N, 0, A)[rows] for t in range(H1)], 1)
            return perturbed_margin(lg, g, float(spec.actor_dist.unimix_ratio))[..., None]

        adv_ = compare_indices(p_act[rows][..., None], z["imag_action"].astype(np.int64)[..., None], amargin,
                               "imagined actions vs reference")
        idv = idv | adv_
    else:
        assert_close(iact[rows], z["imag_action"], 1e-4, 1e-4, "imag_action vs reference", mask=idv[..., None])
    report["ref_imag_rows_flipped"] = int(idv.any(1).sum())
    assert_close(ifeat[rows][..., SK::max(1, spec.D // 4)], z["imag_deter"], 1e-4, 1e-4, "imag_deter vs reference",
                 mask=idv[..., None])
    rows_ok = ~idv.any(1)
    assert_close(p_ret[rows], z["imag_ret"], 1e-3, 1e-3, "imag_ret vs reference", mask=~rows_ok[:, None])
    wm_flip, ac_flip = bool(dv.any()), bool(dv.any() or idv.any())
    if not ac_flip:
        assert_close(ag._last["rret"].detach().cpu().numpy(), z["replay_ret"], 1e-3, 1e-3, "replay_ret vs reference")
        assert_close(ag.return_ema.ema_vals.cpu().numpy(), z["ema_vals"], 1e-3, 1e-5, "ema_vals vs reference")
    bad = []
    for k in losses:
        got, ref = float(mets[f"loss/{k}"]), float(z[f"m_loss/{k}"])
        rel = abs(got - ref) / max(abs(ref), 1e-6)
        report[f"ref_rel_{k}"] = rel
        if rel > _loss_tol(k, wm_flip, ac_flip) and abs(got - ref) > 1e-5:
            bad.append((k, got, ref, rel))
    assert not bad, (bad, report)
    wm = [k for k in losses if k in WM_KEYS]
    sc = {k: float(ag._loss_scales[k]) for k in wm}
    wm_got = sum(sc[k] * float(mets[f"loss/{k}"]) for k in wm)
    wm_ref = sum(sc[k] * float(z[f"m_loss/{k}"]) for k in wm)
    report["ref_wm_loss_rel_err"] = abs(wm_got - wm_ref) / abs(wm_ref)
    fv, fd = (5e-2, 5e-2) if ac_flip else (2e-4, 2e-3)
    report["ref_param_tolerance"] = "widened (near-tie flip vs reference)" if ac_flip else "strict"
    worst = 0.0
    for k in spec.shapes:
        idx = sample_idx(k, got_v[k].size)
        vmax = float(z[f"v_{k}__max"])
        v_ref = z[f"v_{k}__s"].astype(np.float64)
        assert_close(got_v[k][idx], v_ref, 2e-2, fv * vmax + 1e-30, f"exp_avg_sq {k} vs reference")
        vn = float(z[f"v_{k}__n"])
        assert abs(np.linalg.norm(got_v[k]) - vn) <= (2e-2 if not ac_flip else 5e-2) * vn + 1e-30, k
        d_ref = z[f"p_{k}__s"].astype(np.float64) - params[k].reshape(-1)[idx].astype(np.float64)
        dmax = np.abs(got_dp[k]).max()
        tiny = np.sqrt(np.maximum(v_ref, 0)) < 1e-2 * np.sqrt(vmax)
        assert_close(got_dp[k][idx], d_ref, 2e-2, fd * dmax + 4 * ulp(z[f"p_{k}__s"]), f"parameter step {k} vs reference",
                     mask=tiny)
        dn = float(z[f"dp_{k}__n"])
        worst = max(worst, abs(np.linalg.norm(got_dp[k]) - dn) / max(dn, 1e-30))
    report["ref_worst_step_norm_rel"] = worst
    assert worst <= (2e-2 if not ac_flip else 5e-2), report
    print(name, report)
    if not REPORT_DIR:
        return
    os.makedirs(REPORT_DIR, exist_ok=True)
    with open(os.path.join(REPORT_DIR, f"{name}.json"), "w") as f:
        json.dump(report, f, indent=1, sort_keys=True)
