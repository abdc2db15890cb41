"""GPU: the item-sharded hybrid recommender and two-tower scorer (SURVEY §8e,
rows "Scoring" and "Hybrid fusion top-k"; the per-user work they batch and
shard is src/hybrid_system.py:57-75,108 and src/two_tower_model.py:136-146)
run by TWO ranks on one GPU through the real HIP kernels: shard offsets as
global-id bases, the C2 min / max all-reduce of device tensors, the C3
all-gather of the per-shard candidates and the keyed merge
(hrec_topk_f64_keyed). gloo carries the device tensors here (RCCL needs one
GPU per rank; the driver's 8-GPU runs use it).

Every configuration must return exactly (bit for bit) what one rank returns
over the whole item set:
  * "straddle": the split in the middle, with tied item pairs (identical ALS
    factor rows and tower vectors) on both sides of the boundary, ranked into
    the top-k so the tie order (smaller global id first) decides the cut;
  * "small": rank 0 holds 3 items and top_k = 5 exceeds that shard;
  * "empty": rank 1 holds no items.
Precisions: ShardedRecommender "exact" (JVM-exact ALS + f32 Dot), "bf16"
pruned (hrec_hybrid_prune_minmax / _topk; top_k > 8: hrec_hybrid_scores) and
"bf16" unfused (hrec_hybrid_scores + hrec_fuse_rows_topk); ShardedScorer
(hrec_dot_topk) on f32 and bf16 operands.
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N_USERS, N_ITEMS, K, KP, D, B = 300, 5000, 32, 32, 24, 40
CONFIGS = [("exact", "plain", {}), ("bf16", "pruned", {}), ("bf16", "unfused", {"pruned": False})]


def make_data(split):
    """Deterministic inputs (same on every rank); tie pairs straddle `split`
    and score above every other item for every user."""
    rng = np.random.default_rng(2024)
    U = np.zeros((N_USERS, KP), np.float32)
    U[:, :K] = rng.normal(size=(N_USERS, K))
    U[:, 0] = np.abs(U[:, 0]) + 0.5
    V = np.zeros((N_ITEMS, KP), np.float32)
    V[:, :K] = rng.normal(size=(N_ITEMS, K)) * 0.5
    uvec = rng.normal(size=(B, D)).astype(np.float32)
    uvec[:, 0] = np.abs(uvec[:, 0]) + 0.5
    ivec = (rng.normal(size=(N_ITEMS, D)) * 0.5).astype(np.float32)
    for j in range(3):
        a, b = split - 3 + j, split + j
        if 0 <= a < N_ITEMS and 0 <= b < N_ITEMS:
            for M in (V, ivec):
                M[a] = 0.0
                M[a, 0] = 40.0 + j  # pair j: items a and b tie for every user
                M[b] = M[a]
    rows = rng.choice(N_USERS, B, replace=False).astype(np.int64)
    return U, V, uvec, ivec, rows


def run_shard(U, V, uvec, ivec, rows, lo, hi, world, rank, group, top_k):
    """One rank's calls over item rows [lo, hi). Returns {name: (idx, val)}."""
    from src import _hrec
    from src.recommend import ShardedRecommender, ShardedScorer

    dev = torch.device("cuda", 0)
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    dU, duvec, drows = T(U), T(uvec), T(rows)
    V_loc, iv_loc = T(V[lo:hi]), T(ivec[lo:hi])
    Vt_loc = _hrec.transpose(V_loc) if hi > lo else V_loc.t().contiguous()
    out = {}
    for prec, tag, kw in CONFIGS:
        rec = ShardedRecommender(dU, Vt_loc, iv_loc, lo, K, world=world, rank=rank, group=group,
                                 precision=prec, V_local=V_loc if prec == "bf16" else None, **kw)
        for als_wins in (True, False):
            idx, val = rec.recommend(drows, duvec, als_wins, top_k)
            out[f"rec_{prec}_{tag}_{als_wins}"] = (idx.cpu().numpy(), val.double().cpu().numpy())
    for dt in (torch.float32, torch.bfloat16):
        iv_op = _hrec.dot_operand(iv_loc, dt, 32) if hi > lo else torch.zeros((0, 32), dtype=dt, device=dev)
        sc = ShardedScorer(iv_op, lo, world=world, rank=rank, group=group)
        idx, val = sc.topk(_hrec.dot_operand(duvec, dt, 32), top_k)
        out[f"dot_{str(dt).split('.')[-1]}"] = (idx.cpu().numpy(), val.double().cpu().numpy())
    torch.cuda.synchronize()
    return out


def _worker(rank, world, port, split, top_k, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        U, V, uvec, ivec, rows = make_data(split)
        lo, hi = (0, split) if rank == 0 else (split, N_ITEMS)
        q.put((rank, run_shard(U, V, uvec, ivec, rows, lo, hi, world, rank, dist.group.WORLD, top_k)))
        dist.barrier()
    except BaseException as e:  # report instead of leaving the parent waiting
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,split,top_k", [("straddle", N_ITEMS // 2, 5), ("small", 3, 5),
                                               ("empty", N_ITEMS, 5), ("straddle_k10", N_ITEMS // 2, 10)])
def test_two_ranks_match_one_rank(device, case, split, top_k):
    import torch.multiprocessing as mp

    U, V, uvec, ivec, rows = make_data(split)
    ref = run_shard(U, V, uvec, ivec, rows, 0, N_ITEMS, 1, 0, None, top_k)
    if case.startswith("straddle"):
        # the ties are in the top-k and break on the smaller global id
        idx = ref["rec_exact_plain_True"][0]
        pair = [split - 3 + 2, split + 2]
        assert np.all(idx[:, 0] == pair[0]) and np.all(idx[:, 1] == pair[1])
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, split, top_k, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=150) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    for r in range(2):
        assert not isinstance(res[r], str), res[r]
        assert procs[r].exitcode == 0
    for name, (i_ref, v_ref) in ref.items():
        for r in range(2):
            i_got, v_got = res[r][name]
            np.testing.assert_array_equal(i_got, i_ref, err_msg=f"{case} {name} rank {r}")
            np.testing.assert_array_equal(v_got, v_ref, err_msg=f"{case} {name} rank {r}")


# ------------------------------------------- ALSModel.train under torchrun
def _als_frame():
    """A power-law frame (skewed degrees: the nnz-balanced shards differ
    from equal-count ones), duplicates kept, non-contiguous raw ids."""
    import pandas as pd

    rng = np.random.default_rng(77)
    n_u, n_i, nnz = 1500, 900, 40_000
    pu = 1 / (np.arange(n_u) + 1.0) ** 0.6
    pi = 1 / (np.arange(n_i) + 1.0) ** 0.6
    u = rng.choice(n_u, nnz, p=pu / pu.sum()) * 3 + 11
    i = rng.choice(n_i, nnz, p=pi / pi.sum()) * 7 + 5
    return pd.DataFrame({"userId": u, "itemId": i, "average_review_rating": rng.integers(0, 19, nnz),
                         "manufacturer_id": 0, "category_id": 0, "price": 1.0})


def _als_worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from src.als_model import ALSModel

        m = ALSModel(rank=24, max_iter=4, reg_param=0.1, seed=9)
        assert m.train(_als_frame()) is True
        s = m.predict_for_user(int(m.model.user_ids[5]), [int(x) for x in m.model.item_ids[:50]])
        q.put((rank, (m.model.U.cpu().numpy(), m.model.V.cpu().numpy(), [v for _, v in s], m.ingest_peak_bytes)))
        dist.barrier()
    except BaseException as e:
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_als_model_train_two_ranks_matches_one(device):
    """ALSModel.train under an initialised 2-rank world
    (the reference's caller under torchrun, src/als_model.py:43-66) ingests
    its slice of the frame only (src/als_ingest.py: global id encoding, rows
    exchanged to their owners), shards users and items (nnz-balanced parts,
    4 user chunks per rank, chunked all-gathers through the HIP
    half-sweeps) and every rank ends with the factors of the one-rank fit,
    bit for bit; predict_for_user serves the same scores on every rank; the
    ingest's device peak per rank is at most 0.6 of the one-rank ingest's."""
    import torch.multiprocessing as mp

    from src.als_model import ALSModel

    m = ALSModel(rank=24, max_iter=4, reg_param=0.1, seed=9)
    assert m.train(_als_frame()) is True
    U1, V1 = m.model.U.cpu().numpy(), m.model.V.cpu().numpy()
    peak1 = m.ingest_peak_bytes
    s1 = [v for _, v in m.predict_for_user(int(m.model.user_ids[5]), [int(x) for x in m.model.item_ids[:50]])]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_als_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=150) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    for r in range(2):
        assert not isinstance(res[r], str), res[r]
        assert procs[r].exitcode == 0
        U, V, sc, peak = res[r]
        np.testing.assert_array_equal(U, U1)
        np.testing.assert_array_equal(V, V1)
        assert sc == s1
        # the sharded ingest holds about half the device memory
        # of the one-rank ingest (its slice, exchange buffers and own rows)
        assert peak <= 0.6 * peak1, (r, peak, peak1)
