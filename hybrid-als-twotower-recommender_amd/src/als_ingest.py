"""Sharded ratings ingest for ALSModel.train under W > 1 ranks (SURVEY §8(e)
and §8(f) row 1; the reference's ingest is Spark's ALS.fit input handling at
/root/reference/src/als_model.py:51-62: integer ids -> dense indices, the
ratings blocked by user and by item).

Every rank is handed the same frame (torchrun calls train on each rank).
Rank r uploads only its contiguous 1/W slice of the frame's rows and builds
only its own CSR (user) and CSC (item) rows:

  1. id ranges: one all-reduce (MAX over [-min, max] of users and items);
  2. ids -> dense codes: each rank encodes its slice on the device
     (hrec_encode_ids), the slices' distinct ids are all-gathered (sizes
     first) and encoded again: the sorted distinct ids of the whole frame,
     exactly numpy.unique's; a slice's codes are remapped through
     searchsorted positions;
  3. degrees: per-code rating counts, all-reduced (SUM) -> the nnz-balanced
     RowLayouts DeviceALS uses (the same bounds a one-process build gives);
  4. exchange: each rating goes to the rank owning its user row (CSR) and to
     the one owning its item row (CSC) — all_to_all_single of the row codes,
     column codes and rating bits (int32 columns), stably grouped by
     destination, so a destination receives the ratings in frame order;
  5. each rank builds its rows with hrec_coo_to_csr (a row's entries in input
     order) at the layout's local slots (parts in chunk order, each padded to
     cs rows) — bit for bit shard_for_layout of the whole matrix.

Device memory per rank: the slice, the exchange buffers and the rank's own
rows — about 1/W of the one-process ingest (tests/test_gpu_multirank.py
asserts the peak). `ops` (encode_ids, coo_to_csr) defaults to libhrec; the
CPU tests inject numpy stand-ins to pin the orchestration under gloo.
"""
import numpy as np
import torch
import torch.distributed as dist

from .als_engine import RowLayout
from .synthetic import DeviceCSR


class _HrecIngestOps:
    @staticmethod
    def encode_ids(ids, id_range):
        from . import _hrec

        return _hrec.encode_ids(ids, id_range)

    @staticmethod
    def coo_to_csr(rows, cols, vals, n_rows):
        from . import _hrec

        return _hrec.coo_to_csr(rows, cols, vals, int(n_rows), alias=True)  # the exchanged columns are private


def _to_comm(t, group):
    """gloo moves host tensors; RCCL device tensors."""
    return t.cpu() if dist.get_backend(group) == "gloo" else t


def _all_gather_varlen(x, world, group):
    """Every rank's 1-D x (lengths may differ), concatenated in rank order."""
    dev = x.device
    n = torch.tensor([x.numel()], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(_to_comm(n, group)) for _ in range(world)]
    dist.all_gather(ns, _to_comm(n, group), group=group)
    ns = [int(v.item()) for v in ns]
    m = max(max(ns), 1)
    pad = torch.zeros(m, dtype=x.dtype, device=dev)
    pad[: x.numel()] = x
    got = [torch.zeros_like(_to_comm(pad, group)) for _ in range(world)]
    dist.all_gather(got, _to_comm(pad, group), group=group)
    return torch.cat([g[:c].to(dev) for g, c in zip(got, ns)])


def _global_codes(ids, id_range, world, group, ops):
    """(sorted distinct ids of every rank's slice, this slice's int32 codes)."""
    uq, codes = ops.encode_ids(ids, id_range)
    allq = _all_gather_varlen(uq, world, group)
    guq, _ = ops.encode_ids(allq, id_range)
    pos = torch.searchsorted(guq, uq).to(torch.int32)
    return guq, torch.index_select(pos, 0, codes) if codes.numel() else codes


def _part(codes, layout):
    """int32 part index of every code: part c·W + r holds [bounds[p],
    bounds[p+1]); empty parts share a bound with the next, and
    searchsorted(right) lands on the last part starting there."""
    bounds = torch.as_tensor(layout.bounds, dtype=torch.int32, device=codes.device)
    return torch.searchsorted(bounds, codes, right=True, out_int32=True) - 1


def _local_rows(codes, layout, world):
    """This rank's local row of each of its codes (int32): chunk c of the
    rank at rows [c·cs, (c+1)·cs)."""
    p = _part(codes, layout)
    bounds = torch.as_tensor(layout.bounds, dtype=torch.int32, device=codes.device)
    return torch.div(p, world, rounding_mode="floor") * layout.cs + (codes - torch.index_select(bounds, 0, p))


def _exchange(cols_in, dest, world, group):
    """all_to_all_single of each int32 column to `dest`, stable: the result is
    in source-rank order, each source's entries in their input order. One
    boolean mask per destination (masked_select keeps order): no int64 index
    arrays beside the ratings."""
    dev = dest.device
    masks = [dest == d for d in range(world)]
    counts = torch.stack([m.sum() for m in masks]).to(torch.int64)
    rc = torch.empty_like(_to_comm(counts, group))
    dist.all_to_all_single(rc, _to_comm(counts, group), group=group)
    s_split, r_split = counts.cpu().tolist(), rc.cpu().tolist()
    out = []
    for c in cols_in:
        send = torch.cat([torch.masked_select(c, m) for m in masks])
        recv = torch.empty(sum(r_split), dtype=torch.int32, device=dev)
        r = _to_comm(recv, group)
        dist.all_to_all_single(r, _to_comm(send, group), r_split, s_split, group=group)
        del send
        out.append(r.to(dev))
    return out


def _side(rows_g, cols_g, vals, layout, n_cols, world, rank, group, ops):
    """This rank's rows (parts in chunk order, padded to cs) of one side."""
    dest = _part(rows_g, layout) % world
    r_rows, r_cols, r_vals = _exchange([rows_g, cols_g, vals.view(torch.int32)], dest, world, group)
    del dest
    local = _local_rows(r_rows, layout, world)
    del r_rows
    r_vals = r_vals.view(torch.float32)
    n_rows = layout.cs * layout.chunks
    indptr, indices, values = ops.coo_to_csr(local.to(torch.int32), r_cols, r_vals, n_rows)
    return DeviceCSR(indptr, indices, values, layout.part_rows(rank)[0][0], n_rows, int(n_cols))


def frame_fingerprint(users, items, ratings):
    """int64 [5]: length and wrapped sums of the id / rating bits — the same
    frame on every rank or train refuses (a rank's slice of another frame
    would fit a model no rank was given)."""
    r = np.ascontiguousarray(ratings, dtype=np.float32).view(np.int32).astype(np.int64)
    with np.errstate(over="ignore"):
        return np.array([len(users), users.sum(dtype=np.int64), items.sum(dtype=np.int64), r.sum(dtype=np.int64),
                         (users * 31 + items).sum(dtype=np.int64)], dtype=np.int64)


def check_same_frame(fp, dev, group):
    t = torch.as_tensor(fp, device=dev)
    both = torch.cat([t, -t])
    c = _to_comm(both, group)
    dist.all_reduce(c, op=dist.ReduceOp.MAX, group=group)
    c = c.to(dev)
    if not torch.equal(c[: len(fp)], -c[len(fp):]):
        raise ValueError("ALSModel.train: the ranks of the world were given different frames")


def sharded_ingest(users_h, items_h, ratings_h, world, rank, group, chunks, dev, ops=None):
    """-> (user_ids np int64, item_ids np int64, csr shard, csc shard,
    user RowLayout, item RowLayout). users_h / items_h int64 and ratings_h
    f32 host arrays: the WHOLE frame (identical on every rank)."""
    ops = ops or _HrecIngestOps
    n = len(users_h)
    lo, hi = rank * n // world, (rank + 1) * n // world
    u = torch.as_tensor(users_h[lo:hi]).to(dev)
    i = torch.as_tensor(items_h[lo:hi]).to(dev)
    v = torch.as_tensor(np.ascontiguousarray(ratings_h[lo:hi], dtype=np.float32)).to(dev)
    # 1. global id ranges (empty slices contribute nothing)
    big = np.iinfo(np.int64).min
    loc = [-int(u.min()) if u.numel() else big, int(u.max()) if u.numel() else big,
           -int(i.min()) if i.numel() else big, int(i.max()) if i.numel() else big]
    rng = _to_comm(torch.tensor(loc, dtype=torch.int64, device=dev), group)
    dist.all_reduce(rng, op=dist.ReduceOp.MAX, group=group)
    rng = rng.tolist()
    u_range, i_range = (-rng[0], rng[1]), (-rng[2], rng[3])
    # 2. dense codes over the whole frame's distinct ids
    user_ids, cu = _global_codes(u, u_range, world, group, ops)
    item_ids, ci = _global_codes(i, i_range, world, group, ops)
    del u, i
    n_u, n_i = int(user_ids.numel()), int(item_ids.numel())
    # 3. degrees -> the nnz-balanced layouts
    deg = torch.cat([torch.bincount(cu.long(), minlength=n_u), torch.bincount(ci.long(), minlength=n_i)])
    d = _to_comm(deg, group)
    dist.all_reduce(d, op=dist.ReduceOp.SUM, group=group)
    d = d.cpu().numpy()
    ulay = RowLayout.balanced(d[:n_u], world, chunks)
    ilay = RowLayout.balanced(d[n_u:], world, 1)
    del deg, d
    # 4-5. this rank's rows of both sides
    csr = _side(cu, ci, v, ulay, n_i, world, rank, group, ops)
    csc = _side(ci, cu, v, ilay, n_u, world, rank, group, ops)
    return user_ids.cpu().numpy(), item_ids.cpu().numpy(), csr, csc, ulay, ilay
