"""Device ALS engine: the explicit-feedback ALS fit of Spark 3.5.1 that the
reference calls at src/als_model.py:52-62, on MI355X.

Per iteration (Spark ALS.train [ext]): item factors are solved from the
user factors, then user factors from the new item factors — each a
half-sweep (K1, hrec_als_half_sweep) over a CSR shard. With W ranks the
dst rows of each side are split into W equal contiguous shards (the last
padded with empty rows); after each half-sweep the shards are replicated
with one RCCL all-gather (torch.distributed, backend "nccl" = RCCL over
xGMI) so every rank holds the full source matrix for the next half-sweep.
"""
import math

import torch
import torch.distributed as dist

from . import _hrec
from .synthetic import DeviceCSR


def padded_k(k):
    """Leading dimension of the factor storage (padding columns stay 0)."""
    if k <= 16:
        return 16
    if k <= 32:
        return 32
    if k <= 64:
        return 64
    raise ValueError(f"rank {k} > 64 is not supported by the f64 half-sweep kernel")


def shard_range(n, world, rank):
    """Equal contiguous shards of ceil(n/world) rows (rank r's global rows)."""
    per = math.ceil(n / world) if n else 0
    return rank * per, per


class DeviceALS:
    """Holds one rank's CSR shard (user rows), CSC shard (item rows) and the
    replicated factor matrices."""

    def __init__(self, n_users, n_items, rank_k, reg_param, user_csr: DeviceCSR,
                 item_csc: DeviceCSR, world=1, rank=0, group=None, accum_mode=0, sweep=None):
        self.n_users, self.n_items = int(n_users), int(n_items)
        self.k = int(rank_k)
        self.kp = padded_k(self.k)
        self.reg = float(reg_param)
        self.user_csr, self.item_csc = user_csr, item_csc
        self.world, self.rank, self.group = int(world), int(rank), group
        self.accum_mode = int(accum_mode)
        # the half-sweep launcher (K1); tests inject the CPU oracle here to
        # exercise the sharding/all-gather logic on gloo without a GPU
        self.sweep = sweep or _hrec.als_half_sweep
        dev = user_csr.indptr.device
        self.u_per = user_csr.n_rows
        self.i_per = item_csc.n_rows
        if self.world > 1:
            assert user_csr.row_begin == self.rank * self.u_per
            assert item_csc.row_begin == self.rank * self.i_per
        # Replicated factors, padded to world * per rows for the all-gather.
        self.U = torch.zeros((self.u_per * self.world, self.kp), dtype=torch.float32, device=dev)
        self.V = torch.zeros((self.i_per * self.world, self.kp), dtype=torch.float32, device=dev)
        if self.world > 1:
            self.U_local = torch.zeros((self.u_per, self.kp), dtype=torch.float32, device=dev)
            self.V_local = torch.zeros((self.i_per, self.kp), dtype=torch.float32, device=dev)
        else:
            self.U_local, self.V_local = self.U, self.V

    # -------------------------------------------------------------- init
    def init_user_factors(self, seed):
        """Spark-style init of the user side (the item init is never read in
        explicit mode: items are solved first)."""
        _hrec.als_init_factors(seed, 0, self.n_users, self.k, self.kp, self.U)

    def set_user_factors(self, U0):
        """Inject initial user factors ([n_users, k] float32, any device)."""
        self.U.zero_()
        self.U[: self.n_users, : self.k].copy_(torch.as_tensor(U0, dtype=torch.float32))

    # ------------------------------------------------------------- sweeps
    def _gather(self, full, local):
        if self.world > 1:
            dist.all_gather_into_tensor(full, local, group=self.group)

    def item_half_sweep(self):
        self.sweep(self.item_csc.indptr, self.item_csc.indices, self.item_csc.values,
                   self.U, self.k, self.reg, self.V_local, self.accum_mode)
        self._gather(self.V, self.V_local)

    def user_half_sweep(self):
        self.sweep(self.user_csr.indptr, self.user_csr.indices, self.user_csr.values,
                   self.V, self.k, self.reg, self.U_local, self.accum_mode)
        self._gather(self.U, self.U_local)

    def epoch(self):
        """One Spark iteration: items from users, then users from items."""
        self.item_half_sweep()
        self.user_half_sweep()

    def fit(self, max_iter):
        for _ in range(int(max_iter)):
            self.epoch()

    @property
    def user_factors(self):
        return self.U[: self.n_users, : self.k]

    @property
    def item_factors(self):
        return self.V[: self.n_items, : self.k]
