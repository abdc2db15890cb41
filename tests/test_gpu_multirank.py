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
(one-launch hrec_hybrid_scores) and "bf16" fused (hrec_hybrid_minmax /
hrec_hybrid_topk); ShardedScorer (hrec_dot_topk) on f32 and bf16 operands.
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N_USERS, N_ITEMS, K, KP, D, B = 300, 5000, 32, 32, 24, 40
CONFIGS = [("exact", False), ("bf16", False), ("bf16", True)]


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
    for prec, fused in CONFIGS:
        rec = ShardedRecommender(dU, Vt_loc, iv_loc, lo, K, world=world, rank=rank, group=group,
                                 precision=prec, V_local=V_loc if prec == "bf16" else None, fused=fused)
        for als_wins in (True, False):
            idx, val = rec.recommend(drows, duvec, als_wins, top_k)
            out[f"rec_{prec}_{'fused' if fused else 'plain'}_{als_wins}"] = (idx.cpu().numpy(),
                                                                           val.double().cpu().numpy())
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
