"""HBM-resident replay buffer with the reference's API (utils/buffer.py:6-58), no torchrl.

Storage: one tensor per key, laid out (capacity_T, env_num, ...) in device memory (the reference's
LazyTensorStorage(ndim=2) layout). `sample()` draws B slices of L+1 consecutive steps that stay inside one
episode (SliceSampler(traj_key="episode", strict_length=True)), returns data[:, 1:] with the action shifted one
step back (buffer.py:40), the stored latent of step 0 as `initial`, and the (time, env) indices for
`update()` (latent write-back, buffer.py:44-53). Sampling is a device gather: no host round trip per update
once the valid-start table is built (it is rebuilt lazily after new transitions arrive).
torchrl's exact random slice order is not reproduced (parity unpinned); its semantics are.
"""
from __future__ import annotations

import torch


class Buffer:
    def __init__(self, config, device=None, seed=0):
        self.device = torch.device(device or config.device)
        self.storage_device = torch.device(getattr(config, "storage_device", self.device))
        self.batch_size = int(config.batch_size)
        self.batch_length = int(config.batch_length)
        self.max_size = int(float(config.max_size))
        self.num_eps = 0
        self._store = None
        self._t = 0  # rows written (time steps); ring position = _t % cap
        self._dirty = True
        self._starts = None
        self._gen = torch.Generator(device=self.storage_device)
        self._gen.manual_seed(int(seed))
        self._seed, self._draws = int(seed), 0  # device storage: picks from the Philox stream (sd_replay_pick)

    def _alloc(self, td):
        E = next(iter(td.values())).shape[0]
        self.env_num = E
        self.cap = max(self.max_size // E, self.batch_length + 1)
        self._store = {k: torch.zeros((self.cap,) + tuple(v.shape), dtype=v.dtype, device=self.storage_device)
                       for k, v in td.items()}

    def add_transition(self, data):
        """data: dict of (E, ...) tensors (one env step for every env)."""
        if self._store is None:
            self._alloc(data)
        pos = self._t % self.cap
        for k, v in data.items():
            if k not in self._store:
                self._store[k] = torch.zeros((self.cap,) + tuple(v.shape), dtype=v.dtype, device=self.storage_device)
            self._store[k][pos].copy_(v)
        self._t += 1
        self._dirty = True

    def add_sequence(self, data):
        """Bulk insert: dict of (T, E, ...) tensors."""
        T = next(iter(data.values())).shape[0]
        if self._store is None:
            self._alloc({k: v[0] for k, v in data.items()})
        for i in range(0, T):
            pos = (self._t + i) % self.cap
            for k, v in data.items():
                self._store[k][pos].copy_(v[i])
        self._t += T
        self._dirty = True

    def _build_starts(self):
        L1 = self.batch_length + 1
        n = min(self._t, self.cap)
        if n < L1:
            raise RuntimeError("not enough data to sample")
        first = (self._t - n) % self.cap  # oldest row
        order = (torch.arange(n, device=self.storage_device) + first) % self.cap  # chronological rows
        valid = torch.ones(n - L1 + 1, self.env_num, dtype=torch.bool, device=self.storage_device)
        if "episode" in self._store:
            ep = self._store["episode"][order].reshape(n, self.env_num)
            for d in range(1, L1):
                valid &= ep[d:n - L1 + 1 + d] == ep[: n - L1 + 1]
        idx = valid.nonzero()  # (V, 2): chronological start, env
        if idx.shape[0] == 0:
            raise RuntimeError("no valid slices")
        self._starts = torch.stack([order[idx[:, 0]], idx[:, 1]], 1)
        self._dirty = False

    def _pick(self):
        """B slice indices into the valid-start table: a device Philox draw on GPU storage (one launch, no torch RNG
        kernel), torch's generator on CPU storage."""
        B, V = self.batch_size, self._starts.shape[0]
        if self.storage_device.type != "cuda":
            return torch.randint(0, V, (B,), device=self.storage_device, generator=self._gen)
        from . import _native as nat
        from . import kernels as K
        pick = torch.empty(B, dtype=torch.int64, device=self.storage_device)
        nat.call("sd_replay_pick", self._seed & 0xFFFFFFFFFFFFFFFF, self._draws & 0xFFFFFFFF, V, B, K.p(pick), K.stream())
        self._draws += 1
        return pick

    def sample(self):
        if self._dirty:
            self._build_starts()
        B, L1 = self.batch_size, self.batch_length + 1
        pick = self._pick()
        st = self._starts[pick]
        t_idx = (st[:, :1] + torch.arange(L1, device=self.storage_device)[None]) % self.cap  # (B, L+1)
        e_idx = st[:, 1:2].expand(B, L1)
        sample = {k: v[t_idx, e_idx].to(self.device, non_blocking=True) for k, v in self._store.items()}
        initial = (sample["stoch"][:, 0], sample["deter"][:, 0]) if "stoch" in sample else None
        data = {k: v[:, 1:] for k, v in sample.items() if k not in ("stoch", "deter")}
        data["action"] = sample["action"][:, :-1]  # action is 1 step back (buffer.py:40)
        index = [t_idx[:, 1:], e_idx[:, 1:]]
        return data, index, initial

    # ---------------------------------------------------------------- fused device path (one launch each way)
    def _slice_keys(self, pairs):
        from . import _native as nat
        ks = nat.SliceKeys()
        for i, (store, batch, steps, shift) in enumerate(pairs):
            if batch.dtype != store.dtype or not batch.is_contiguous() or batch.device != store.device:
                raise ValueError("slice batch buffer must match the storage dtype / device and be contiguous")
            ks.k[i].storage, ks.k[i].batch = store.data_ptr(), batch.data_ptr()
            ks.k[i].row_bytes = store[0, 0].numel() * store.element_size()
            ks.k[i].steps, ks.k[i].shift = steps, shift
        ks.n = len(pairs)
        return ks

    def sample_into(self, dst, dst_initial=None):
        """sample() written straight into caller-owned buffers (dst: the data dict's keys, (B, L, ...) each;
        dst_initial: (stoch (B, S, K), deter (B, D))), every key in one gather launch (sd_replay_slices). Returns
        the write-back index, which update() turns into one scatter launch."""
        import ctypes

        from . import _native as nat
        from . import kernels as K
        if self._dirty:
            self._build_starts()
        B, L = self.batch_size, self.batch_length
        pick = self._pick()
        pairs = [(v, dst[k], L, 0 if k == "action" else 1) for k, v in self._store.items()
                 if k not in ("stoch", "deter")]
        if dst_initial is not None and "stoch" in self._store:
            pairs += [(self._store["stoch"], dst_initial[0], 1, 0), (self._store["deter"], dst_initial[1], 1, 0)]
        t_idx = torch.empty(B, L, dtype=torch.int64, device=self.storage_device)
        e_idx = torch.empty(B, L, dtype=torch.int64, device=self.storage_device)
        starts = self._starts.contiguous()
        ks = self._slice_keys(pairs)
        nat.call("sd_replay_slices", ctypes.addressof(ks), K.p(starts), K.p(pick), B, L, self.cap, self.env_num,
                 K.p(t_idx), K.p(e_idx), 0, K.stream())
        index = [t_idx, e_idx]
        self._last = (index, pick, starts)
        return index

    def update(self, index, stoch, deter):
        """Write posterior latents back to the sampled positions (buffer.py:44-53)."""
        last = getattr(self, "_last", None)
        if last is not None and index is last[0] and "stoch" in self._store and "deter" in self._store:
            import ctypes

            from . import _native as nat
            from . import kernels as K
            _, pick, starts = last
            B, L = self.batch_size, self.batch_length
            ks = self._slice_keys([(self._store["stoch"], stoch.contiguous(), L, 1),
                                   (self._store["deter"], deter.contiguous(), L, 1)])
            nat.call("sd_replay_slices", ctypes.addressof(ks), K.p(starts), K.p(pick), B, L, self.cap,
                     self.env_num, None, None, 1, K.stream())
            self._last = None
            return
        t_idx, e_idx = index
        keep = self._last_writer(t_idx, e_idx).reshape(-1)
        ti, ei = t_idx.reshape(-1)[keep], e_idx.reshape(-1)[keep]
        if "stoch" in self._store:
            self._store["stoch"][ti, ei] = stoch.reshape(-1, *stoch.shape[2:]).to(self.storage_device)[keep]
        if "deter" in self._store:
            self._store["deter"][ti, ei] = deter.reshape(-1, deter.shape[-1]).to(self.storage_device)[keep]

    def _last_writer(self, t_idx, e_idx):
        """(B, L) bool: False where a later slice (larger b) writes the same storage row. Overlapping slices make the
        write-back hit one row several times; index_put with duplicate indices picks an arbitrary one on the GPU, so
        the slice with the largest b wins here (a sequential scatter in row order), as in sd_replay_slices."""
        B, L = t_idx.shape
        start, env = t_idx[:, :1], e_idx[:, :1]  # slices are consecutive (mod cap) from their first row
        cover = ((t_idx[:, :, None] - start.reshape(1, 1, B)) % self.cap < L) & \
            (env.reshape(B, 1, 1) == env.reshape(1, 1, B))
        later = torch.arange(B, device=t_idx.device)
        cover &= (later.reshape(1, 1, B) > later.reshape(B, 1, 1))
        return ~cover.any(-1)

    def count(self):
        if self._store is None:
            return 0
        return min(self._t, self.cap) * self.env_num
