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
import os

import torch
import torch.distributed as dist

from . import _hrec
from .synthetic import DeviceCSR


# f64 sources up to this size (the MI355X's 256 MB MALL holds them; larger
# ones are gathered in f32): the c2 user side (51 MB) qualifies, its item
# side (512 MB) does not
SRC64_MAX_BYTES = int(os.environ.get("HREC_ALS_SRC64_MB", "128")) << 20


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


class RowLayout:
    """How one side's rows (users or items) sit in the replicated factor
    buffer across W ranks and C chunks per rank ("partitioned by
    nnz-balanced contiguous ranges"). Part p = c·W + r (chunk c of rank r)
    owns the contiguous global rows [bounds[p], bounds[p+1]) and stores them
    at buffer rows [p·cs, p·cs + count_p): every part has cs slots, so each
    chunk's RCCL all-gather moves equal-sized shards (the padding rows stay
    zero and are never referenced).

    equal(): count-balanced parts with bounds[p] = p·cs — buffer row ==
    global row (the CSR ids need no remap). balanced(): bounds chosen on the
    row costs nnz + row_cost (Gramian work per rating + a per-row solve
    term), so skewed degree distributions (power-law items) give every rank
    the same work; the shards' column ids are then remapped to buffer rows
    (hrec_remap_i32) once, at setup."""

    def __init__(self, n, world, chunks, bounds):
        self.n, self.world, self.chunks = int(n), int(world), int(chunks)
        self.bounds = [int(b) for b in bounds]
        if len(self.bounds) != self.world * self.chunks + 1 or self.bounds[0] != 0 or self.bounds[-1] != self.n:
            raise ValueError("RowLayout: bounds must run 0 .. n over world * chunks parts")
        counts = [b - a for a, b in zip(self.bounds, self.bounds[1:])]
        if min(counts) < 0:
            raise ValueError("RowLayout: bounds must be non-decreasing")
        self.cs = max(1, max(counts))

    @classmethod
    def equal(cls, n, world, chunks=1):
        per = math.ceil(n / world) if n else 0
        cs = math.ceil(per / chunks) if per else 0
        return cls(n, world, chunks, [min(p * cs, n) for p in range(world * chunks + 1)])

    @classmethod
    def balanced(cls, row_nnz, world, chunks=1, row_cost=128):
        """Contiguous parts of (near) equal cost, cost(row) = nnz + row_cost."""
        import numpy as np

        w = np.asarray(row_nnz, dtype=np.float64) + float(row_cost)
        n, P = len(w), world * chunks
        cum = np.concatenate([[0.0], np.cumsum(w)])
        # part p starts at the first row whose preceding cost reaches p/P of the total
        starts = np.searchsorted(cum, cum[-1] * np.arange(P + 1) / P, side="left")
        starts = np.minimum(np.maximum.accumulate(starts), n)
        starts[0], starts[-1] = 0, n
        return cls(n, world, chunks, starts.tolist())

    @property
    def identity(self):
        """Buffer row == global row for every real row."""
        return all(self.bounds[p] == min(p * self.cs, self.n) for p in range(len(self.bounds)))

    @property
    def slots(self):
        return self.world * self.chunks * self.cs

    def part_rows(self, rank):
        """[(global row_begin, count)] of this rank's chunks, in chunk order."""
        return [(self.bounds[c * self.world + rank], self.bounds[c * self.world + rank + 1] -
                 self.bounds[c * self.world + rank]) for c in range(self.chunks)]

    def positions(self):
        """int32 [n]: buffer row of each global row."""
        import numpy as np

        pos = np.empty(self.n, dtype=np.int32)
        for p in range(len(self.bounds) - 1):
            a, b = self.bounds[p], self.bounds[p + 1]
            pos[a:b] = p * self.cs + np.arange(b - a, dtype=np.int32)
        return pos


def shard_for_layout(csr, layout, rank):
    """This rank's shard of a whole-matrix CSR (DeviceCSR over every row,
    global column ids) under `layout`: its parts in chunk order, each part's
    rows followed by empty rows up to layout.cs (the layout's padded slots),
    indices / values copied (DeviceALS remaps the copy's column ids in place).
    Pure torch ops, any device."""
    ips, ixs, vs, off = [csr.indptr[:1] * 0], [], [], 0
    ip_all = csr.indptr
    for b, cnt in layout.part_rows(rank):
        lo, hi = int(ip_all[b]), int(ip_all[b + cnt])
        ip = torch.full((layout.cs,), hi - lo, dtype=torch.int64, device=ip_all.device)
        ip[:cnt] = ip_all[b + 1: b + cnt + 1] - lo
        ips.append(ip + off)
        ixs.append(csr.indices[lo:hi])
        vs.append(csr.values[lo:hi])
        off += hi - lo
    return DeviceCSR(torch.cat(ips), torch.cat(ixs).clone(), torch.cat(vs).clone(), layout.part_rows(rank)[0][0],
                     layout.cs * layout.chunks, csr.n_cols)


def process_group():
    """(world, rank, group) of an initialised torch.distributed world with
    more than one rank, else (1, 0, None). HREC_ALS_SHARD=0 keeps one rank's
    fit unsharded even then."""
    if os.environ.get("HREC_ALS_SHARD", "1") == "0" or not dist.is_available() or not dist.is_initialized():
        return 1, 0, None
    w = dist.get_world_size()
    return (w, dist.get_rank(), dist.group.WORLD) if w > 1 else (1, 0, None)


class DeviceALS:
    """Holds one rank's CSR shard (user rows), CSC shard (item rows) and the
    replicated factor matrices."""

    def __init__(self, n_users, n_items, rank_k, reg_param, user_csr: DeviceCSR,
                 item_csc: DeviceCSR, world=1, rank=0, group=None, accum_mode=0, sweep=None, chunks=1,
                 item_chunks=1, user_layout=None, item_layout=None, remap=None):
        """user_layout / item_layout (RowLayout): the shards' row layout;
        default RowLayout.equal(n, world, chunks). With a non-identity layout
        the shards are this rank's parts padded to cs rows each (see
        synthetic.generate_layout) with GLOBAL column ids; they are remapped
        here (remap, default hrec_remap_i32) to rows of the other side's
        buffer."""
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
        # f64 copies of sources that stay in the on-chip caches (the device
        # sweep only): hrec_als_half_sweep_src64, same results, no per-row
        # conversion in the gather
        self._src64_ok = sweep is None and self.kp == 64 and self.accum_mode == 0
        self._s64 = None
        dev = user_csr.indptr.device
        self.u_per = user_csr.n_rows
        self.i_per = item_csc.n_rows
        # row chunks per side (user side: `chunks`, item side: `item_chunks`)
        self.u_chunks = int(chunks) if self.world > 1 else 1
        self.i_chunks = int(item_chunks) if self.world > 1 else 1
        self.u_layout = user_layout or RowLayout.equal(self.n_users, self.world, self.u_chunks)
        self.i_layout = item_layout or RowLayout.equal(self.n_items, self.world, self.i_chunks)
        for lay, ch, per, csr in ((self.u_layout, self.u_chunks, self.u_per, user_csr),
                                  (self.i_layout, self.i_chunks, self.i_per, item_csc)):
            if lay.world != self.world or lay.chunks != ch or per != ch * lay.cs:
                raise ValueError("DeviceALS: shard rows do not match the row layout")
            if self.world > 1 and csr.row_begin != lay.part_rows(self.rank)[0][0]:
                raise ValueError("DeviceALS: shard does not start at the layout's first row for this rank")
        self.u_cs, self.i_cs = self.u_layout.cs, self.i_layout.cs
        self._u_pos = self._i_pos = None  # global row -> buffer row (non-identity layouts)
        if not self.u_layout.identity or not self.i_layout.identity:
            remap = remap or _hrec.remap_i32
            self._u_pos = torch.as_tensor(self.u_layout.positions(), device=dev)
            self._i_pos = torch.as_tensor(self.i_layout.positions(), device=dev)
            for csr, lay, pos in ((user_csr, self.i_layout, self._i_pos), (item_csc, self.u_layout, self._u_pos)):
                if lay.identity or csr.col_layout is lay:
                    continue  # global ids are buffer rows / already remapped for this layout
                if csr.col_layout is not None:
                    raise ValueError("DeviceALS: shard ids were remapped to another layout")
                remap(csr.indices, pos)  # user rows hold item ids, item rows user ids
                csr.col_layout = lay
        chunked = max(self.u_chunks, self.i_chunks) > 1
        self.comm = torch.cuda.Stream(device=dev) if chunked and dev.type == "cuda" else None
        # Replicated factors in the layouts' padded buffers (world * per rows).
        self.U = torch.zeros((self.u_layout.slots, self.kp), dtype=torch.float32, device=dev)
        self.V = torch.zeros((self.i_layout.slots, self.kp), dtype=torch.float32, device=dev)
        if self.world > 1:
            self.U_local = torch.zeros((self.u_per, self.kp), dtype=torch.float32, device=dev)
            self.V_local = torch.zeros((self.i_per, self.kp), dtype=torch.float32, device=dev)
        else:
            self.U_local, self.V_local = self.U, self.V

    # -------------------------------------------------------------- init
    def init_user_factors(self, seed):
        """Spark-style init of the user side (the item init is never read in
        explicit mode: items are solved first). Counter-based per global row,
        so every layout holds the same vectors."""
        if self._u_pos is None:
            _hrec.als_init_factors(seed, 0, self.n_users, self.k, self.kp, self.U)
            return
        lay = self.u_layout
        for p in range(len(lay.bounds) - 1):
            a, b = lay.bounds[p], lay.bounds[p + 1]
            if b > a:
                _hrec.als_init_factors(seed, a, b - a, self.k, self.kp, self.U[p * lay.cs: p * lay.cs + b - a])

    def set_user_factors(self, U0):
        """Inject initial user factors ([n_users, k] float32, any device)."""
        self.U.zero_()
        U0 = torch.as_tensor(U0, dtype=torch.float32).to(self.U.device)
        if self._u_pos is None:
            self.U[: self.n_users, : self.k].copy_(U0)
        else:
            self.U[self._u_pos.long(), : self.k] = U0

    # ------------------------------------------------------------- sweeps
    def _gather(self, full, local):
        if self.world > 1:
            dist.all_gather_into_tensor(full, local, group=self.group)

    def _src64(self, src):
        """The f64 copy of `src` for the half-sweep, or None when the source
        is larger than SRC64_MAX_BYTES (it would stream from HBM at twice
        the bytes: the f32 gather is faster there)."""
        if not self._src64_ok or src.numel() * 8 > SRC64_MAX_BYTES:
            return None
        if self._s64 is None or self._s64.numel() < src.numel():
            self._s64 = torch.empty(src.numel(), dtype=torch.float64, device=src.device)
        out = self._s64[: src.numel()].view(src.shape)
        return _hrec.f32_to_f64(src, out)

    def _sweep(self, csr, src, local, full, cs, chunks):
        """One half-sweep of this rank's rows + replication of the result."""
        s64 = self._src64(src)
        extra = {} if s64 is None else {"src64": s64}
        if chunks == 1:
            self.sweep(csr.indptr, csr.indices, csr.values, src, self.k, self.reg, local, self.accum_mode, **extra)
            self._gather(full, local)
            return
        W = self.world
        compute = torch.cuda.current_stream() if self.comm is not None else None
        for c in range(chunks):
            rows = slice(c * cs, (c + 1) * cs)
            self.sweep(csr.indptr[c * cs: (c + 1) * cs + 1], csr.indices, csr.values, src, self.k, self.reg,
                       local[rows], self.accum_mode, **extra)
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

    def compute_only_epoch(self):
        """The epoch's half-sweep kernels alone (this rank's rows, the same
        chunk launches, no all-gathers: the replicated buffers are not
        updated) — what an epoch would cost if the collectives were free
        (bench.py: epoch time minus this = collective time not hidden)."""
        for csr, src, local, cs, chunks in ((self.item_csc, self.U, self.V_local, self.i_cs, self.i_chunks),
                                            (self.user_csr, self.V, self.U_local, self.u_cs, self.u_chunks)):
            s64 = self._src64(src)
            extra = {} if s64 is None else {"src64": s64}
            for c in range(chunks):
                self.sweep(csr.indptr[c * cs: (c + 1) * cs + 1], csr.indices, csr.values, src, self.k, self.reg,
                           local[c * cs: (c + 1) * cs], self.accum_mode, **extra)

    def epoch(self):
        """One Spark iteration: items from users, then users from items."""
        self.item_half_sweep()
        self.user_half_sweep()

    def fit(self, max_iter):
        for _ in range(int(max_iter)):
            self.epoch()

    def user_rows(self, ids):
        """Buffer rows of U for global user ids (a device int64 tensor)."""
        return ids if self._u_pos is None else self._u_pos[ids].to(torch.int64)

    def item_factor_rows(self, start, count):
        """[count, kp] item factors of global items [start, start + count)."""
        if self._i_pos is None:
            return self.V[start: start + count]
        return self.V[self._i_pos[start: start + count].long()]

    @property
    def user_factors(self):
        """[n_users, k] in global row order."""
        if self._u_pos is None:
            return self.U[: self.n_users, : self.k]
        return self.U[self._u_pos.long(), : self.k]

    @property
    def item_factors(self):
        if self._i_pos is None:
            return self.V[: self.n_items, : self.k]
        return self.V[self._i_pos.long(), : self.k]
