"""Counter-based noise for sampling sites (oracle side; mirrored bit-exactly by safe-dreamer_amd/csrc/philox.h).

The reference draws its sampling noise from torch's global RNG: Gumbel noise in F.gumbel_softmax
(`-empty_like().exponential_().log()`, used by OneHotDist.rsample, world_model/distributions.py:33) and
N(0,1) in Normal.rsample (bounded_normal, distributions.py:217-222). Global-RNG streams cannot be matched
across CPU/GPU or across a data-parallel split, so this build defines noise as a pure function of
(seed, stream, step, element index) and the golden generator injects exactly this noise into the reference.

  word  = Philox4x32-10(counter=(q_lo, q_hi, step, stream), key=(seed_lo, seed_hi))[w]
  u     = ((word >> 8) + 0.5) * 2**-24                       in (0, 1), exact
  gumbel= float32(-log(-log(u)))                              evaluated in float64
  normal= float32(sqrt(-2 log u1) * cos(2*pi*u2))             evaluated in float64
For gumbel: q = idx >> 2, w = idx & 3.  For normal: q = idx, (u1, u2) from words 0, 1.
Streams: OBS=1 (posterior sample in RSSM.observe), IMG=2 (prior sample in img_step during _imagine),
ACT=3 (actor sample during _imagine), POLICY=4 (act() train-mode sample).
Element indices are GLOBAL (row index in the un-sharded batch), so data-parallel shards draw the same noise.
"""
import numpy as np

STREAM_OBS = 1
STREAM_IMG = 2
STREAM_ACT = 3
STREAM_POLICY = 4
STREAM_POLICY_ACT = 5  # the action sample of Dreamer.act (the posterior sample there uses STREAM_POLICY)
STREAM_AUG = 6  # random_translate shifts (r2dreamer aug; DreamerPro's doubled batch)
STREAM_OBS_AUG = 7  # DreamerPro's posterior scan over the augmented (2B) batch

_M0 = np.uint64(0xD2511F53)
_M1 = np.uint64(0xCD9E8D57)
_W0 = np.uint32(0x9E3779B9)
_W1 = np.uint32(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10. All inputs uint32 arrays (broadcastable). Returns 4 uint32 arrays."""
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint32) for x in (c0, c1, c2, c3))
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    with np.errstate(over="ignore"):
        for r in range(10):
            p0 = _M0 * c0.astype(np.uint64)
            p1 = _M1 * c2.astype(np.uint64)
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo0 = (p0 & _MASK).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & _MASK).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            if r < 9:
                k0 = np.uint32(k0 + _W0)
                k1 = np.uint32(k1 + _W1)
    return c0, c1, c2, c3


def _key(seed):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return seed & 0xFFFFFFFF, seed >> 32


def _uniform(word):
    return ((word >> np.uint32(8)).astype(np.float64) + 0.5) * (2.0 ** -24)


def gumbel(seed, stream, step, idx):
    """float32 Gumbel(0,1) noise for global element indices `idx` (int64 array)."""
    idx = np.asarray(idx, dtype=np.int64)
    q = (idx >> 2).astype(np.uint64)
    w = (idx & 3).astype(np.int64)
    k0, k1 = _key(seed)
    out = philox4x32_10((q & _MASK).astype(np.uint32), (q >> np.uint64(32)).astype(np.uint32),
                        np.uint32(step), np.uint32(stream), k0, k1)
    word = np.choose(w, out)
    u = _uniform(word)
    return (-np.log(-np.log(u))).astype(np.float32)


def normal(seed, stream, step, idx):
    """float32 N(0,1) noise (Box-Muller) for global element indices `idx`."""
    idx = np.asarray(idx, dtype=np.int64).astype(np.uint64)
    k0, k1 = _key(seed)
    out = philox4x32_10((idx & _MASK).astype(np.uint32), (idx >> np.uint64(32)).astype(np.uint32),
                        np.uint32(step), np.uint32(stream), k0, k1)
    u1 = _uniform(out[0])
    u2 = _uniform(out[1])
    return (np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)).astype(np.float32)


def gumbel_block(seed, stream, step, rows, row_offset, width):
    """Noise for a (rows, width) block whose first row is global row `row_offset`."""
    idx = (np.arange(rows, dtype=np.int64)[:, None] + row_offset) * width + np.arange(width, dtype=np.int64)[None]
    return gumbel(seed, stream, step, idx)


def normal_block(seed, stream, step, rows, row_offset, width):
    idx = (np.arange(rows, dtype=np.int64)[:, None] + row_offset) * width + np.arange(width, dtype=np.int64)[None]
    return normal(seed, stream, step, idx)


def uniform_int(seed, stream, step, idx, n):
    """integer in [0, n) from the word gumbel() would use for idx (augmentation shifts)."""
    idx = np.asarray(idx, dtype=np.int64)
    q = (idx >> 2).astype(np.uint64)
    w = (idx & 3).astype(np.int64)
    k0, k1 = _key(seed)
    out = philox4x32_10((q & _MASK).astype(np.uint32), (q >> np.uint64(32)).astype(np.uint32),
                        np.uint32(step), np.uint32(stream), k0, k1)
    v = np.floor(_uniform(np.choose(w, out)) * n).astype(np.int64)
    return np.minimum(v, n - 1)


def aug_shifts(seed, rows, row_offset, T, pad, same_across_time):
    """random_translate shifts (dreamer.py:864-868) for slice rows row_offset..: (rows, T, 2) ints, (x, y)."""
    n = 2 * pad + 1
    b = np.arange(rows, dtype=np.int64)[:, None, None] + row_offset
    t = np.arange(T, dtype=np.int64)[None, :, None]
    ax = np.arange(2, dtype=np.int64)[None, None, :]
    idx = b * 2 + ax + 0 * t if same_across_time else (b * T + t) * 2 + ax
    return uniform_int(seed, STREAM_AUG, 0, idx, n)
