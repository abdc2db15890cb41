"""Device ALS engine: the explicit-feedback ALS fit of Spark 3.5.1 that the
reference calls at src/als_model.py:52-62, on MI355X.

Per iteration (Spark ALS.train [ext]): item factors are solved from the
user factors, then user factors from the new item factors — each a
half-sweep (K1, hrec_als_half_sweep) over a CSR shard. With W ranks the
dst rows of each side are split into W equal shards (padded with empty
rows); after each half-sweep the shards are replicated with RCCL
all-gathers (torch.distributed, backend "nccl" = RCCL over xGMI) so every
rank holds the full source matrix for the next half-sweep.

With C > 1 chunks a side's shard is C chunks of cs rows, interleaved with
the other ranks' (rank r owns global rows [c·W·cs + r·cs, +cs) for
c < C): the half-sweep runs chunk by chunk and each chunk's all-gather —
contiguous in the replicated matrix — is issued on a side stream as soon as
its kernel finishes, so C−1 of the C all-gathers overlap the next chunk's
compute. Chunking pays on the user side (many short rows, the large factor
matrix); the item side's few long rows would lose more to per-launch tails
than its small all-gather costs, so the two sides take separate counts.
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
    for kp in (64, 96, 128, 192, 256):  # > 64: one workgroup per row (csrc/als_wide.hip)
        if k <= kp:
            return kp
    raise ValueError(f"rank {k} > 256 is not supported by the half-sweep kernels")


def shard_range(n, world, rank):
    """Equal contiguous shards of ceil(n/world) rows (rank r's global rows)."""
    per = math.ceil(n / world) if n else 0
    return rank * per, per


def shard_chunks(n, world, rank, chunks):
    """Chunk-interleaved shard: ([(global_begin, cs)] for c < chunks, cs).
    chunks == 1 is shard_range's contiguous shard."""
    per = math.ceil(n / world) if n else 0
    cs = math.ceil(per / chunks) if per else 0
    return [(c * world * cs + rank * cs, cs) for c in range(chunks)], cs


class DeviceALS:
    """Holds one rank's CSR shard (user rows), CSC shard (item rows) and the
    replicated factor matrices."""

    def __init__(self, n_users, n_items, rank_k, reg_param, user_csr: DeviceCSR,
                 item_csc: DeviceCSR, world=1, rank=0, group=None, accum_mode=0, sweep=None, chunks=1,
                 item_chunks=1):
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
        # row chunks per side (user side: `chunks`, item side: `item_chunks`)
        self.u_chunks = int(chunks) if self.world > 1 else 1
        self.i_chunks = int(item_chunks) if self.world > 1 else 1
        self.u_cs, self.i_cs = self.u_per, self.i_per
        if self.world > 1:
            ur, self.u_cs = shard_chunks(self.n_users, self.world, self.rank, self.u_chunks)
            ir, self.i_cs = shard_chunks(self.n_items, self.world, self.rank, self.i_chunks)
            assert self.u_per == self.u_chunks * self.u_cs and self.i_per == self.i_chunks * self.i_cs
            assert user_csr.row_begin == ur[0][0] and item_csc.row_begin == ir[0][0]
        chunked = max(self.u_chunks, self.i_chunks) > 1
        self.comm = torch.cuda.Stream(device=dev) if chunked and dev.type == "cuda" else None
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

    def _sweep(self, csr, src, local, full, cs, chunks):
        """One half-sweep of this rank's rows + replication of the result."""
        if chunks == 1:
            self.sweep(csr.indptr, csr.indices, csr.values, src, self.k, self.reg, local, self.accum_mode)
            self._gather(full, local)
            return
        W = self.world
        compute = torch.cuda.current_stream() if self.comm is not None else None
        for c in range(chunks):
            rows = slice(c * cs, (c + 1) * cs)
            self.sweep(csr.indptr[c * cs: (c + 1) * cs + 1], csr.indices, csr.values, src, self.k, self.reg,
                       local[rows], self.accum_mode)
            out = full[c * W * cs: (c + 1) * W * cs]
            if self.comm is None:
                dist.all_gather_into_tensor(out, local[rows], group=self.group)
                continue
            done = torch.cuda.Event()
            done.record(compute)
            with torch.cuda.stream(self.comm):
                self.comm.wait_event(done)
                dist.all_gather_into_tensor(out, local[rows], group=self.group)
        if self.comm is not None:
            compute.wait_stream(self.comm)

    def item_half_sweep(self):
        self._sweep(self.item_csc, self.U, self.V_local, self.V, self.i_cs, self.i_chunks)

    def user_half_sweep(self):
        self._sweep(self.user_csr, self.V, self.U_local, self.U, self.u_cs, self.u_chunks)

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
