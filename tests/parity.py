"""Parity helpers shared by the GPU tests (test infrastructure; imports the CPU oracle only as the checker).

Latent-index rule (BASELINE.json north_star, SURVEY §7 "RNG parity"): sampled indices must match the reference
bit for bit, except at near-ties, where the top-2 margin of the Gumbel-perturbed unimix logits is below
`MARGIN` (an argmax flip there is expected from last-bit differences between two fp32 evaluations). A flip
changes the rest of that row's trajectory (the next step's input), so only each row's FIRST mismatch is judged
and the row is excluded from later comparisons (`diverged` mask).
"""
import numpy as np
import torch

from oracle import noise as nz
from oracle.ref_cpu import unimix_logits

MARGIN = 1e-5


def perturbed_margin(logits, g, unimix):
    """top-2 gap of log p̃ + g over the last axis (distributions.py:16-33, F.gumbel_softmax's argmax)."""
    x = unimix_logits(torch.as_tensor(np.asarray(logits, np.float32)), unimix) + torch.as_tensor(g)
    top2 = torch.topk(x, 2, dim=-1).values
    return (top2[..., 0] - top2[..., 1]).numpy()


def post_margins(logit, seed, unimix, stream=nz.STREAM_OBS, row_offset=0):
    """Margins of the posterior samples of RSSM.observe: logit (B, T, S, K) -> (B, T, S)."""
    B, T, S, K = logit.shape
    g = np.stack([nz.gumbel_block(seed, stream, t, B, row_offset, S * K).reshape(B, S, K) for t in range(T)], 1)
    return perturbed_margin(logit, g, unimix)


def imag_margins(prior_logit, seed, unimix, row_offset=0):
    """Margins of the imagined prior samples: prior_logit (N, H, S, K) of img_step t (feat index t + 1)."""
    N, H, S, K = prior_logit.shape
    g = np.stack([nz.gumbel_block(seed, nz.STREAM_IMG, t, N, row_offset, S * K).reshape(N, S, K)
                  for t in range(H)], 1)
    return perturbed_margin(prior_logit, g, unimix)


def compare_indices(got, ref, margin_fn, what, max_row_frac=0.02):
    """got / ref: (rows, T, S) int. margin_fn() -> (rows, T, S) margins at the REFERENCE's logits (lazy: only
    evaluated when a mismatch exists). Asserts every row's first mismatch is a near-tie and that at most
    `max_row_frac` of the rows diverge. Returns the (rows, T) bool mask of steps at or after a row's first flip."""
    got = np.asarray(got)
    ref = np.asarray(ref)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    neq = got != ref
    rows, T = neq.shape[:2]
    diverged = np.zeros((rows, T), bool)
    if not neq.any():
        return diverged
    m = margin_fn()
    step_bad = neq.reshape(rows, T, -1).any(-1)
    bad = []
    for r in np.nonzero(step_bad.any(1))[0]:
        t = int(np.argmax(step_bad[r]))
        diverged[r, t:] = True
        sites = np.nonzero(neq.reshape(rows, T, -1)[r, t])[0]
        worst = float(m.reshape(rows, T, -1)[r, t, sites].max())
        if worst >= MARGIN:
            bad.append((int(r), t, sites.tolist(), worst))
    assert not bad, f"{what}: index flips that are not near-ties (row, step, latents, margin): {bad[:8]}"
    frac = diverged.any(1).mean()
    assert frac <= max_row_frac, f"{what}: {frac:.3%} of rows flipped at a near-tie (bound {max_row_frac:.0%})"
    return diverged


def ulp(x):
    return np.spacing(np.abs(np.asarray(x, np.float32))).astype(np.float64)


def bound_ratio(got, ref, rtol, atol, mask=None):
    """max over elements of |got - ref| / (atol + rtol |ref|): the fraction of assert_close's bound used (<= 1 passes)"""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    bound = np.broadcast_to(np.asarray(atol, np.float64), ref.shape) + rtol * np.abs(ref)
    r = np.abs(got - ref) / np.maximum(bound, 1e-300)
    if mask is not None:
        r = np.where(mask, 0.0, r)
    return float(r.max()) if r.size else 0.0


def assert_close(got, ref, rtol, atol, what, mask=None):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    atol = np.broadcast_to(np.asarray(atol, np.float64), ref.shape)
    err = np.abs(got - ref) - (atol + rtol * np.abs(ref))
    if mask is not None:
        err = np.where(mask, -1.0, err)
    i = int(np.argmax(err))
    g, r, a = got.reshape(-1)[i], ref.reshape(-1)[i], atol.reshape(-1)[i]
    assert err.reshape(-1)[i] <= 0, (f"{what}: |{g} - {r}| = {abs(g - r):.3g} > {a:.3g} + {rtol:.3g}*|ref| "
                                     f"(flat index {i})")
