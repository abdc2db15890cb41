"""CPU, world_size 2 (gloo): the multi-GPU ALS path — equal row shards of
users and items, padded shards, one all_gather_into_tensor per half-sweep —
reproduces the unsharded fit bit for bit. The per-row arithmetic is the C
oracle injected as the sweep (the HIP kernel is the same per row on GPU; its
parity is covered by the gpu tests), so this pins the orchestration."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import als as oals
from oracle import build as obuild

N_USERS, N_ITEMS, DENS, K, REG, ITERS, SEED, SEED2 = 103, 57, 0.09, 12, 0.1, 3, 5, 6


def _oracle_sweep(indptr, indices, values, src, k, reg, dst, accum_mode=0):
    out = obuild.half_sweep(indptr.numpy(), indices.numpy(), values.numpy(), src[:, :k].numpy(), k, reg)
    dst.zero_()
    dst[: out.shape[0], :k] = torch.from_numpy(out)


def _shard(n_users, n_items, transposed, world, rank, chunks=1):
    """This rank's (chunk-interleaved) shard, built by the C oracle generator
    range by range and concatenated like synthetic.generate_ranges."""
    from src.als_engine import shard_chunks
    from src.synthetic import DeviceCSR

    total = n_items if transposed else n_users
    ranges, _ = shard_chunks(total, world, rank, chunks)
    ips, ixs, vs, off = [np.zeros(1, np.int64)], [], [], 0
    for r0, cnt in ranges:
        ip, ix, v = obuild.synth_csr(n_users, n_items, DENS, int(transposed), r0, cnt, SEED, SEED2)
        ips.append(ip[1:] + off)
        ixs.append(ix)
        vs.append(v)
        off += len(ix)
    return DeviceCSR(torch.from_numpy(np.concatenate(ips)), torch.from_numpy(np.concatenate(ixs)),
                     torch.from_numpy(np.concatenate(vs)), ranges[0][0], sum(c for _, c in ranges),
                     n_users if transposed else n_items)


def _worker(rank, world, port, U0, q, chunks=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from src.als_engine import DeviceALS

    # user side in `chunks` chunks, item side in chunks - 1 (both layouts mixed)
    ichunks = max(1, chunks - 1)
    eng = DeviceALS(N_USERS, N_ITEMS, K, REG, _shard(N_USERS, N_ITEMS, False, world, rank, chunks),
                    _shard(N_USERS, N_ITEMS, True, world, rank, ichunks), world=world, rank=rank,
                    group=dist.group.WORLD, sweep=_oracle_sweep, chunks=chunks, item_chunks=ichunks)
    eng.set_user_factors(U0)
    eng.fit(ITERS)
    q.put((rank, eng.user_factors.numpy().copy(), eng.item_factors.numpy().copy()))
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,chunks", [(2, 1), (3, 1), (2, 3), (3, 4)])
def test_sharded_als_matches_unsharded(world, chunks):
    """Contiguous shards (chunks=1) and chunk-interleaved shards whose
    per-chunk all-gathers overlap the next chunk's sweep (chunks>1)."""
    rng = np.random.default_rng(0)
    U0 = rng.normal(size=(N_USERS, K)).astype(np.float32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, U0, q, chunks)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=60) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ucsr = obuild.synth_csr(N_USERS, N_ITEMS, DENS, 0, 0, N_USERS, SEED, SEED2)
    icsc = obuild.synth_csr(N_USERS, N_ITEMS, DENS, 1, 0, N_ITEMS, SEED, SEED2)
    U, V = oals.fit(ucsr, icsc, U0, K, REG, ITERS, sweep=obuild.half_sweep)
    for _, Ur, Vr in res:
        np.testing.assert_array_equal(Ur, U)
        np.testing.assert_array_equal(Vr, V)


# ------------------------------------- nnz-balanced shards (skewed degrees)
SK_USERS, SK_ITEMS, SK_NNZ, SK_K = 2000, 1500, 60000, 8


def _skewed_csr(transposed):
    """A power-law (Zipf 0.5) user x item matrix with duplicates kept as
    separate terms (Spark keeps them), as one CSR over users (or items);
    entries of a row in input order."""
    rng = np.random.default_rng(3)
    pu = 1 / (np.arange(SK_USERS) + 1.0) ** 0.5
    pi = 1 / (np.arange(SK_ITEMS) + 1.0) ** 0.5
    u = rng.choice(SK_USERS, SK_NNZ, p=pu / pu.sum())
    i = rng.choice(SK_ITEMS, SK_NNZ, p=pi / pi.sum())
    r = rng.integers(0, 19, SK_NNZ).astype(np.float32)
    rows, cols, n = (i, u, SK_ITEMS) if transposed else (u, i, SK_USERS)
    order = np.argsort(rows, kind="stable")
    indptr = np.zeros(n + 1, np.int64)
    indptr[1:] = np.cumsum(np.bincount(rows, minlength=n))
    return indptr, cols[order].astype(np.int32), r[order]


def _layout_shard(csr, layout, rank, n_cols):
    """This rank's parts of a host CSR, each padded with empty rows to cs."""
    from src.synthetic import DeviceCSR

    indptr, indices, values = csr
    ips, ixs, vs, off = [np.zeros(1, np.int64)], [], [], 0
    for b, cnt in layout.part_rows(rank):
        lo, hi = indptr[b], indptr[b + cnt]
        ip = np.full(layout.cs, hi - lo, np.int64)
        ip[:cnt] = indptr[b + 1: b + cnt + 1] - lo
        ips.append(ip + off)
        ixs.append(indices[lo:hi])
        vs.append(values[lo:hi])
        off += hi - lo
    return DeviceCSR(torch.from_numpy(np.concatenate(ips)), torch.from_numpy(np.concatenate(ixs).copy()),
                     torch.from_numpy(np.concatenate(vs)), layout.part_rows(rank)[0][0], layout.cs * layout.chunks,
                     n_cols)


def _cpu_remap(x, table):
    x.copy_(table[x.long()])


def _balanced_worker(rank, world, port, U0, q, chunks):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from src.als_engine import DeviceALS, RowLayout

    ucsr, icsc = _skewed_csr(False), _skewed_csr(True)
    ulay = RowLayout.balanced(np.diff(ucsr[0]), world, chunks)
    ilay = RowLayout.balanced(np.diff(icsc[0]), world, 1)
    eng = DeviceALS(SK_USERS, SK_ITEMS, SK_K, REG, _layout_shard(ucsr, ulay, rank, SK_ITEMS),
                    _layout_shard(icsc, ilay, rank, SK_USERS), world=world, rank=rank, group=dist.group.WORLD,
                    sweep=_oracle_sweep, chunks=chunks, item_chunks=1, user_layout=ulay, item_layout=ilay,
                    remap=_cpu_remap)
    eng.set_user_factors(U0)
    eng.fit(2)
    q.put((rank, eng.user_factors.numpy().copy(), eng.item_factors.numpy().copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,chunks", [(2, 1), (3, 3)])
def test_nnz_balanced_shards_match_unsharded(world, chunks):
    """users / items partitioned into contiguous ranges of equal
    cost (nnz + a per-row solve term) on a power-law matrix — every rank's
    cost within 5 % of every other's (equal-count shards: > 15 % apart),
    nnz alone balanced the same way within 5 %; the sharded fit (padded
    parts, remapped ids, chunked all-gathers) equals the unsharded one bit for
    bit."""
    from src.als_engine import RowLayout

    for transposed, n, ch in ((False, SK_USERS, chunks), (True, SK_ITEMS, 1)):
        deg = np.diff(_skewed_csr(transposed)[0])
        for rc in (128, 0):
            lay, eq = RowLayout.balanced(deg, world, ch, row_cost=rc), RowLayout.equal(n, world, ch)

            def per(L):
                return [sum(float((deg[a:a + c] + rc).sum()) for a, c in L.part_rows(r)) for r in range(world)]

            assert max(per(lay)) / min(per(lay)) <= 1.05
            assert max(per(eq)) / min(per(eq)) > 1.15
    rng = np.random.default_rng(1)
    U0 = rng.normal(size=(SK_USERS, SK_K)).astype(np.float32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_balanced_worker, args=(r, world, port, U0, q, chunks)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    U, V = oals.fit(_skewed_csr(False), _skewed_csr(True), U0, SK_K, REG, 2, sweep=obuild.half_sweep)
    for _, Ur, Vr in res:
        np.testing.assert_array_equal(Ur, U)
        np.testing.assert_array_equal(Vr, V)


def test_shard_for_layout_matches_host_shard():
    """als_engine.shard_for_layout (what ALSModel.train cuts out of the
    whole-frame CSR under W > 1) == the host shard builder of these tests,
    for balanced chunked layouts, incl. empty parts (more parts than rows)."""
    from src.als_engine import RowLayout, shard_for_layout
    from src.synthetic import DeviceCSR

    for transposed in (False, True):
        ip, ix, v = _skewed_csr(transposed)
        n_cols = SK_USERS if transposed else SK_ITEMS
        full = DeviceCSR(torch.from_numpy(ip), torch.from_numpy(ix), torch.from_numpy(v), 0, len(ip) - 1, n_cols)
        for world, chunks in ((2, 1), (3, 4), (5, 3)):
            lay = RowLayout.balanced(np.diff(ip), world, chunks)
            for r in range(world):
                a, b = shard_for_layout(full, lay, r), _layout_shard((ip, ix, v), lay, r, n_cols)
                assert torch.equal(a.indptr, b.indptr) and torch.equal(a.indices, b.indices)
                assert torch.equal(a.values, b.values)
                assert (a.row_begin, a.n_rows, a.n_cols) == (b.row_begin, b.n_rows, b.n_cols)
                assert a.indices.data_ptr() != full.indices.data_ptr()  # remapped in place later: a copy
    tiny = DeviceCSR(torch.tensor([0, 2, 3], dtype=torch.int64), torch.tensor([1, 0, 1], dtype=torch.int32),
                     torch.tensor([1.0, 2.0, 3.0]), 0, 2, 2)
    lay = RowLayout.balanced([2, 1], 3, 2)
    shards = [shard_for_layout(tiny, lay, r) for r in range(3)]
    assert sum(s.nnz for s in shards) == 3 and all(s.n_rows == lay.cs * 2 for s in shards)


def test_row_layout_positions():
    from src.als_engine import RowLayout

    eq = RowLayout.equal(103, 3, 2)
    assert eq.identity and list(eq.positions()) == list(range(103))
    lay = RowLayout(10, 2, 2, [0, 4, 5, 9, 10])
    assert lay.cs == 4 and not lay.identity and lay.slots == 16
    assert list(lay.positions()) == [0, 1, 2, 3, 4, 8, 9, 10, 11, 12]
    assert lay.part_rows(0) == [(0, 4), (5, 4)] and lay.part_rows(1) == [(4, 1), (9, 1)]


def test_shard_ranges_cover_and_pad():
    from src.als_engine import shard_range

    for n in (1, 7, 100, 1000001):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            per = spans[0][1]
            assert all(s[1] == per for s in spans)
            assert per * w >= n and per == -(-n // w)  # covers [0, n); tail shards padded
            assert [s[0] for s in spans] == [r * per for r in range(w)]


def test_shard_chunks_tile_the_padded_matrix():
    from src.als_engine import shard_chunks, shard_range

    for n in (1, 7, 57, 103, 1000):
        for w in (1, 2, 3, 8):
            for c in (1, 2, 3, 4):
                owned = []
                for r in range(w):
                    ranges, cs = shard_chunks(n, w, r, c)
                    assert len(ranges) == c and all(cnt == cs for _, cnt in ranges)
                    owned += [b + i for b, cnt in ranges for i in range(cnt)]
                # every row of the padded [c*w*cs] matrix owned exactly once
                assert sorted(owned) == list(range(c * w * cs)) and c * w * cs >= n
                if c == 1:
                    assert shard_chunks(n, w, 0, 1)[0][0] == shard_range(n, w, 0)


# ------------------------------------------------ sharded hybrid top-k (C2/C3)
class _CpuOps:
    """CPU stand-ins with the kernels' arithmetic (exact on integer-valued data)."""

    @staticmethod
    def als_scores(U, user_rows, Vt_local, n_local, k):
        s = oals.score_matrix(U[user_rows.numpy(), :k].numpy(), Vt_local[:k, :n_local].numpy().T)
        return torch.from_numpy(s)

    @staticmethod
    def tt_scores(user_vecs, item_vecs_local):
        return torch.from_numpy((user_vecs.numpy().astype(np.float64) @ item_vecs_local.numpy().T.astype(np.float64))
                                .astype(np.float32))

    @staticmethod
    def operand(x, dtype, dk=None):
        return x.to(dtype).to(torch.float32)  # bf16 rounding of the operand, CPU stand-in

    @staticmethod
    def dot_scores(U, V):
        return torch.from_numpy((U.numpy().astype(np.float64) @ V.numpy().T.astype(np.float64)).astype(np.float32))

    @staticmethod
    def rows_minmax(x):
        a = x.numpy()
        return torch.from_numpy(np.stack([np.nanmin(a, axis=1), np.nanmax(a, axis=1)]).astype(np.float32))

    @staticmethod
    def fuse_rows_topk(als, tt, a_mm, t_mm, als_wins, top_k, offset):
        w0, w1 = (0.8, 0.2) if als_wins else (0.2, 0.8)
        out_i, out_v = [], []
        for r in range(als.shape[0]):
            amin, amax = float(a_mm[0, r]), float(a_mm[1, r])
            rng = amax - amin
            rng = 1.0 if rng < 10 * np.finfo(np.float64).eps else rng
            sc = 1.0 / rng
            an = als[r].numpy().astype(np.float64) * sc + (0.0 - amin * sc)
            tmin, tmax = np.float32(t_mm[0, r]), np.float32(t_mm[1, r])
            trng = np.float32(tmax - tmin)
            trng = np.float32(1.0) if trng < np.float32(10) * np.finfo(np.float32).eps else trng
            ts = np.float32(np.float32(1.0) / trng)
            tn = tt[r].numpy() * ts + np.float32(np.float32(0.0) - tmin * ts)
            f = w0 * an + w1 * tn.astype(np.float64)
            order = np.lexsort((np.arange(len(f)), -f))[:top_k]
            out_i.append(order + offset)
            out_v.append(f[order])
        return torch.from_numpy(np.array(out_i)), torch.from_numpy(np.array(out_v))

    @staticmethod
    def topk_keyed(vals, keys, top_k):
        out_i, out_v = [], []
        for v, kk in zip(vals.numpy(), keys.numpy()):
            ok = kk >= 0
            v, kk = v[ok], kk[ok]
            order = np.lexsort((kk, -v))[:top_k]
            out_i.append(kk[order])
            out_v.append(v[order])
        return torch.from_numpy(np.array(out_i)), torch.from_numpy(np.array(out_v))


def _hybrid_data():
    rng = np.random.default_rng(7)
    n_users, n_items, k, d = 12, 101, 8, 6
    U = rng.integers(-3, 4, (n_users, 16)).astype(np.float32)
    V = rng.integers(-3, 4, (n_items, 16)).astype(np.float32)
    uv = rng.integers(-2, 3, (5, d)).astype(np.float32)
    iv = rng.integers(-2, 3, (n_items, d)).astype(np.float32)
    return U, V, uv, iv, k


def _hybrid_run(world, rank, U, V, uv, iv, k, group=None, precision="exact"):
    from src.als_engine import shard_range
    from src.recommend import ShardedRecommender

    i0, per = shard_range(V.shape[0], world, rank)
    Vl = V[i0: i0 + per]
    rec = ShardedRecommender(torch.from_numpy(U), torch.from_numpy(np.ascontiguousarray(Vl.T)),
                             torch.from_numpy(iv[i0: i0 + per]), i0, k, world=world, rank=rank, group=group,
                             ops=_CpuOps, precision=precision,
                             V_local=torch.from_numpy(np.ascontiguousarray(Vl)))
    rows = torch.tensor([0, 3, 5, 7, 11], dtype=torch.int64)
    return [t.numpy() for t in rec.recommend(rows, torch.from_numpy(uv), True, 7)]


def _hybrid_worker(rank, world, port, q, precision="exact"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from src import recommend

    U, V, uv, iv, k = _hybrid_data()
    c0 = recommend.COLLECTIVE_CALLS[0]
    out = _hybrid_run(world, rank, U, V, uv, iv, k, dist.group.WORLD, precision)
    q.put((rank, out, recommend.COLLECTIVE_CALLS[0] - c0))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,precision", [(2, "exact"), (4, "exact"), (24, "exact"), (3, "bf16"),
                                             (24, "bf16")])
def test_sharded_hybrid_topk_matches_single(world, precision):
    U, V, uv, iv, k = _hybrid_data()
    ref_i, ref_v = _hybrid_run(1, 0, U, V, uv, iv, k, precision=precision)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hybrid_worker, args=(r, world, port, q, precision)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=60) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, (gi, gv), calls in res:
        np.testing.assert_array_equal(gi, ref_i)
        np.testing.assert_array_equal(gv, ref_v)
        assert calls == 2  # C2 (one all_reduce) + C3 (one all_gather) per batch


# ------------------------------------------- sharded two-tower top-k (c4, C3)
class _CpuDotOps(_CpuOps):
    @staticmethod
    def dot_topk(user_vecs, item_vecs_local, top_k, offset):
        s = (user_vecs.numpy().astype(np.float64) @ item_vecs_local.numpy().T.astype(np.float64)).astype(np.float32)
        kk = min(top_k, s.shape[1])
        order = np.argsort(-s.astype(np.float64), axis=1, kind="stable")[:, :kk]
        return torch.from_numpy(order + offset), torch.from_numpy(np.take_along_axis(s, order, 1))


def _scorer_data():
    rng = np.random.default_rng(11)
    uv = rng.integers(-3, 4, (6, 8)).astype(np.float32)
    iv = rng.integers(-3, 4, (53, 8)).astype(np.float32)  # integer data: many exact ties
    return uv, iv


def _scorer_run(world, rank, uv, iv, group=None):
    from src.als_engine import shard_range
    from src.recommend import ShardedScorer

    i0, per = shard_range(iv.shape[0], world, rank)
    sc = ShardedScorer(torch.from_numpy(iv[i0: i0 + per]), i0, world=world, rank=rank, group=group, ops=_CpuDotOps)
    i, v = sc.topk(torch.from_numpy(uv), 7)
    return i.numpy(), v.numpy().astype(np.float64)


def test_global_minmax_packs_both_models():
    """C2 packing: [a_min | t_min | -a_max | -t_max] reduced by MIN gives
    both models' global min and max exactly (one rank: the identity), incl.
    the +inf / -inf extremes of an empty shard."""
    from src.recommend import global_minmax

    a = torch.tensor([[1.5, float("inf"), -2.0], [3.0, -float("inf"), -0.0]])
    t = torch.tensor([[-7.0, 0.25, float("inf")], [9.0, 0.5, -float("inf")]])

    class _G:
        pass

    orig = dist.all_reduce
    dist.all_reduce = lambda x, op=None, group=None: x  # world 1: MIN over one rank
    try:
        ga, gt = global_minmax(a, t, _G())
    finally:
        dist.all_reduce = orig
    assert torch.equal(ga, a) and torch.equal(gt, t)


def _scorer_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    uv, iv = _scorer_data()
    q.put((rank, _scorer_run(world, rank, uv, iv, dist.group.WORLD)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 24])
def test_sharded_dot_topk_matches_single(world):
    """Item-sharded two-tower top-k (local top-k with global ids, all_gather,
    keyed merge) == one rank, ties included (ties -> smaller item id); world 24
    leaves some ranks without items."""
    uv, iv = _scorer_data()
    ref_i, ref_v = _scorer_run(1, 0, uv, iv)
    s = uv.astype(np.float64) @ iv.T.astype(np.float64)
    np.testing.assert_array_equal(ref_i, np.argsort(-s, axis=1, kind="stable")[:, :7])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scorer_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, (gi, gv) in res:
        np.testing.assert_array_equal(gi, ref_i)
        np.testing.assert_array_equal(gv, ref_v)


# ------------------------------------------- sharded ingest (ALSModel.train, W > 1)
class _NumpyIngestOps:
    """numpy stand-ins for hrec_encode_ids / hrec_coo_to_csr (numpy.unique;
    a stable sort by row): the device kernels' parity is pinned by the gpu
    tests, these pin the orchestration."""

    @staticmethod
    def encode_ids(ids, id_range):
        u, inv = np.unique(ids.numpy(), return_inverse=True)
        return torch.from_numpy(u.astype(np.int64)), torch.from_numpy(inv.astype(np.int32).reshape(-1))

    @staticmethod
    def coo_to_csr(rows, cols, vals, n_rows):
        r = rows.numpy()
        order = np.argsort(r, kind="stable")
        indptr = np.zeros(n_rows + 1, np.int64)
        indptr[1:] = np.cumsum(np.bincount(r, minlength=n_rows))
        return (torch.from_numpy(indptr), torch.from_numpy(cols.numpy()[order].copy()),
                torch.from_numpy(vals.numpy()[order].copy()))


def _ingest_frame():
    """Skewed degrees, duplicates, non-contiguous raw ids (some only in one
    rank's slice), negative ids."""
    rng = np.random.default_rng(11)
    n_u, n_i, nnz = 700, 300, 9001
    pu = 1 / (np.arange(n_u) + 1.0) ** 0.7
    pi = 1 / (np.arange(n_i) + 1.0) ** 0.7
    u = rng.choice(n_u, nnz, p=pu / pu.sum()) * 5 - 1000
    i = rng.choice(n_i, nnz, p=pi / pi.sum()) * 3 + 7
    r = rng.integers(0, 19, nnz).astype(np.float32) * 0.25
    return u.astype(np.int64), i.astype(np.int64), r


def _ingest_worker(rank, world, port, q, chunks, tamper):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from src.als_ingest import check_same_frame, frame_fingerprint, sharded_ingest

        u, i, r = _ingest_frame()
        if tamper and rank == world - 1:
            r = r.copy()
            r[17] += 1.0
        try:
            check_same_frame(frame_fingerprint(u, i, r), torch.device("cpu"), dist.group.WORLD)
        except ValueError as e:
            q.put((rank, "refused: " + str(e)))
            return
        uid, iid, csr, csc, ulay, ilay = sharded_ingest(u, i, r, world, rank, dist.group.WORLD, chunks,
                                                        torch.device("cpu"), ops=_NumpyIngestOps)
        q.put((rank, (uid, iid, ulay.bounds, ilay.bounds,
                      [(c.indptr.numpy(), c.indices.numpy(), c.values.numpy(), c.row_begin, c.n_rows, c.n_cols)
                       for c in (csr, csc)])))
    finally:
        dist.destroy_process_group()


def _run_ingest(world, chunks, tamper=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ingest_worker, args=(r, world, port, q, chunks, tamper)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=90) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,chunks", [(2, 4), (3, 1), (3, 4)])
def test_sharded_ingest_matches_whole_build(world, chunks):
    """each rank uploads its 1/W slice of the frame, encodes
    ids globally (range all-reduce + all-gathered distinct ids), balances
    rows on the all-reduced degrees and receives its rows' ratings by
    all_to_all — its CSR / CSC parts equal the whole matrix's cut by
    shard_for_layout (ids, layouts, indptr, in-row order, values) exactly."""
    from src.als_engine import RowLayout

    res = _run_ingest(world, chunks)
    u, i, r = _ingest_frame()
    uid, cu = np.unique(u, return_inverse=True)
    iid, ci = np.unique(i, return_inverse=True)
    ops = _NumpyIngestOps
    whole = [ops.coo_to_csr(torch.from_numpy(cu.astype(np.int32)), torch.from_numpy(ci.astype(np.int32)),
                            torch.from_numpy(r), len(uid)),
             ops.coo_to_csr(torch.from_numpy(ci.astype(np.int32)), torch.from_numpy(cu.astype(np.int32)),
                            torch.from_numpy(r), len(iid))]
    lays = [RowLayout.balanced(np.diff(whole[0][0].numpy()), world, chunks),
            RowLayout.balanced(np.diff(whole[1][0].numpy()), world, 1)]
    for rank in range(world):
        g_uid, g_iid, ub, ib, sides = res[rank]
        np.testing.assert_array_equal(g_uid, uid)
        np.testing.assert_array_equal(g_iid, iid)
        assert ub == lays[0].bounds and ib == lays[1].bounds
        for s, (ip, ix, v, row0, n_rows, n_cols) in enumerate(sides):
            want = _layout_shard(tuple(t.numpy() for t in whole[s]), lays[s], rank, (len(iid), len(uid))[s])
            np.testing.assert_array_equal(ip, want.indptr.numpy())
            np.testing.assert_array_equal(ix, want.indices.numpy())
            np.testing.assert_array_equal(v, want.values.numpy())
            assert (row0, n_rows, n_cols) == (want.row_begin, want.n_rows, want.n_cols)


def test_sharded_ingest_refuses_different_frames():
    """the ranks' frames are fingerprinted (length, id and rating
    bit sums) and compared by one all-reduce before any slice is taken."""
    res = _run_ingest(2, 1, tamper=True)
    for rank in range(2):
        assert isinstance(res[rank], str) and res[rank].startswith("refused"), res[rank]
