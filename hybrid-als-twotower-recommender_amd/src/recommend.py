"""Batched hybrid top-k recommendations with the item set sharded across GPUs.

What HybridRecommendationSystem.get_hybrid_recommendations does for one user
(src/hybrid_system.py:95-116: ALS scores and two-tower scores for every
candidate item, per-model MinMaxScaler over all candidates, weighted fusion,
stable top-k) done for a BATCH of users on the device, with the candidate
items split into contiguous shards, one per rank (SURVEY §8e, rows
"Scoring" and "Hybrid fusion top-k"):

  1. local scores: JVM-exact ALS dot (hrec_als_score) and two-tower Dot on
     the matrix cores (hrec_tt_score) for the rank's item shard;
  2. per-row min / max of both (hrec_rows_minmax_f32), made global by ONE
     RCCL all_reduce MIN over [min | -max] of both models (C2) — min and
     max are exact under any grouping;
  3. fusion with the global scaler coefficients + local stable top-k with
     global item ids (hrec_fuse_rows_topk);
  4. ONE RCCL all_gather of the [B, k] candidates, ids and scores in one
     buffer (C3), and a keyed stable top-k merge (hrec_topk_f64_keyed): ties
     break on the global item id, so every world size returns the same items
     and scores as one GPU. Two collectives per batch in all.

ShardedScorer does the same for the two-tower scoring alone (BASELINE c4:
d = 128 embeddings, 50M candidates over 8 GPUs): each rank ranks its item
shard with the fused matrix-core dot + top-k (hrec_dot_topk, global ids via
the shard offset), then C3 + keyed merge as above — the score matrix never
exists on any rank.

The collectives and kernels are injectable (`ops`) so the orchestration can be
exercised with gloo on CPU (tests/test_distributed.py).
"""
import torch
import torch.distributed as dist

from . import _hrec


class DeviceOps:
    """The libhrec implementations of the per-shard steps."""

    @staticmethod
    def als_scores(U, user_rows, Vt_local, n_local, k):
        return _hrec.als_score(U, user_rows, Vt_local, None, n_local, k)

    @staticmethod
    def tt_scores(user_vecs, item_vecs_local):
        return _hrec.tt_score(user_vecs, item_vecs_local)

    @staticmethod
    def dot_topk(user_vecs, item_vecs_local, top_k, offset):
        return _hrec.dot_topk(user_vecs, item_vecs_local, top_k, idx_offset=offset)

    @staticmethod
    def operand(x, dtype, dk=None):
        return _hrec.dot_operand(x, dtype, dk)

    @staticmethod
    def hybrid_exact_items(Vt_local, n_local, k, item_vecs_local):
        """The shard's items prepared for hrec_hybrid_exact_* (the transposed
        ALS factors are the ones hrec_als_score reads)."""
        return _hrec.HybridExactItems(Vt_local, n_local, k, item_vecs_local.contiguous())

    hybrid_exact = staticmethod(_hrec.HybridExact)
    dot_scores = staticmethod(_hrec.dot_scores)
    hybrid_scores = staticmethod(_hrec.hybrid_scores)
    hybrid_prune = staticmethod(_hrec.HybridPrune)
    rows_minmax = staticmethod(_hrec.rows_minmax)
    fuse_rows_topk = staticmethod(_hrec.fuse_rows_topk)
    topk_keyed = staticmethod(_hrec.topk_keyed)


# Batch shapes whose workspaces a recommender keeps (one per shape
# ever seen grew device memory without bound for callers that vary the batch).
WORKSPACE_CACHE = 4


def _lru_get(cache, key):
    """cache: a dict in insertion order = recency order."""
    v = cache.pop(key, None)
    if v is not None:
        cache[key] = v
    return v


def _lru_put(cache, key, value):
    cache[key] = value
    while len(cache) > WORKSPACE_CACHE:
        cache.pop(next(iter(cache)))
    return value


class ShardedRecommender:
    """precision "exact": JVM-exact ALS scores (Spark's f32 mul/add chain) and
    f32 two-tower Dot — the reference's numerics. For top_k <= 8, batches of
    >= 8 users and two-tower widths 32/64/128 the exact path is the pruned one
    (hrec_hybrid_exact_*: both models bounded on the bf16 matrix cores, the
    exact chains only for the item groups the bounds cannot rule out; no
    score matrix in HBM); pruned=False keeps the score matrices
    (als_score + tt_score + rows_minmax + fuse_rows_topk) — the same bits.
    precision "bf16" (BASELINE
    config c5: rank-256 factors and d = 256 towers stored in bf16): both
    models' scores on the bf16 matrix cores (f32 accumulation) from bf16
    copies of the factors / item vectors made once here; pass V_local (the
    shard's ALS item factor rows) instead of Vt_local. For top_k <= 8 the bf16
    path is the pruned one (hrec_hybrid_prune_*: no score matrix in HBM, the
    exact path inside the survivor kernel for the users that need it; one
    shard: hrec_hybrid_prune_local); pruned=False keeps the score
    matrices (hrec_hybrid_scores + hrec_fuse_rows_topk); all three bf16
    paths return the same bits."""

    def __init__(self, U, Vt_local, item_vecs_local, item_offset, k, world=1, rank=0, group=None, ops=None,
                 precision="exact", V_local=None, pruned=True):
        self.U = U                          # [n_users, kp] ALS user factors (replicated)
        self.Vt = Vt_local                  # [kp, ld] transposed ALS item factors of this shard
        self.iv = item_vecs_local           # [n_local, d] two-tower item vectors of this shard
        self.n_local = item_vecs_local.shape[0]
        self.offset = int(item_offset)
        self.k = int(k)
        self.world, self.rank, self.group = int(world), int(rank), group
        self.ops = ops or DeviceOps
        if precision not in ("exact", "bf16"):
            raise ValueError(f"precision must be 'exact' or 'bf16', got {precision!r}")
        self.precision = precision
        self.pruned_exact = False
        if precision == "exact":
            self.pruned_exact = (bool(pruned) and hasattr(self.ops, "hybrid_exact")
                                 and _hrec.exact_dk(self.k, int(item_vecs_local.shape[1])) is not None)
            self.exact_items = None
            if self.pruned_exact and self.n_local > 0:
                self.exact_items = self.ops.hybrid_exact_items(Vt_local, self.n_local, self.k, item_vecs_local)
        if precision == "bf16":
            if V_local is None:
                raise ValueError("precision='bf16' needs V_local (ALS item factor rows of the shard)")
            # one width for both models so the fused kernel can run them together
            self.dk = max(64, _hrec.dot_dk(V_local.shape[1]), _hrec.dot_dk(item_vecs_local.shape[1]))
            self.pruned = bool(pruned) and hasattr(self.ops, "hybrid_prune")
            self.V_op = self.ops.operand(V_local, torch.bfloat16, self.dk)
            self.iv_op = self.ops.operand(item_vecs_local, torch.bfloat16, self.dk)

    def _user_ops(self, user_rows, user_vecs):
        o = self.ops
        return (o.operand(self.U.index_select(0, user_rows), torch.bfloat16, self.dk),
                o.operand(user_vecs, torch.bfloat16, self.dk))

    def _scores(self, user_rows, user_vecs):
        o = self.ops
        if self.precision == "exact":
            return (o.als_scores(self.U, user_rows, self.Vt, self.n_local, self.k),
                    o.tt_scores(user_vecs, self.iv))
        u_als, u_tt = self._user_ops(user_rows, user_vecs)
        return o.dot_scores(u_als, self.V_op), o.dot_scores(u_tt, self.iv_op)

    def _recommend_pruned(self, user_rows, user_vecs, als_wins, top_k):
        """bf16 path without score matrices (hrec_hybrid_prune_*): phase 1 gives
        each user's min / max of both rows (C2 makes them global), phase 2 the
        local top-k from the heavier model's survivors."""
        o = self.ops
        B = int(user_rows.shape[0])
        dev = user_vecs.device
        if self.n_local > 0:
            # one workspace per batch shape, reused across batches (a few shapes kept)
            key = (B, int(top_k), tuple(user_vecs.shape))
            hp = _lru_get(self.__dict__.setdefault("_prune", {}), key)
            if hp is None:
                hp = _lru_put(self._prune, key, o.hybrid_prune(self.U, user_rows, user_vecs, self.V_op, self.iv_op,
                                                               top_k))
            else:
                hp.rebind(user_rows, user_vecs)
            if self.world == 1:  # one shard: both phases in one call (no C2 between them)
                idx, val, _, _ = hp.local(als_wins, self.offset)
                self.last_prune = hp
                return idx, val
            a_mm, t_mm = hp.minmax()
        else:
            inf = float("inf")
            a_mm = torch.tensor([[inf] * B, [-inf] * B], dtype=torch.float32, device=dev)
            t_mm = a_mm.clone()
        if self.world > 1:
            a_mm, t_mm = global_minmax(a_mm, t_mm, self.group)
        if self.n_local > 0:
            idx, val = hp.topk(a_mm, t_mm, als_wins, self.offset)
            self.last_prune = hp
        else:
            idx = torch.empty((B, 0), dtype=torch.int64, device=dev)
            val = torch.empty((B, 0), dtype=torch.float64, device=dev)
        if self.world == 1:
            return idx, val
        return merge_candidates(idx, val, top_k, self.world, self.group, o)

    def _recommend_exact_pruned(self, user_rows, user_vecs, als_wins, top_k):
        """Exact path without score matrices (hrec_hybrid_exact_*): phase 1 +
        the exact extremes, C2, the top-k; one call for one shard."""
        o = self.ops
        B = int(user_rows.shape[0])
        dev = user_vecs.device
        if self.n_local > 0:
            key = (B, int(top_k))
            hx = _lru_get(self.__dict__.setdefault("_hx", {}), key)
            if hx is None:
                hx = _lru_put(self._hx, key, o.hybrid_exact(self.U, user_rows, user_vecs, self.exact_items, top_k))
            else:
                hx.rebind(user_rows, user_vecs)
            self.last_exact = hx
            if self.world == 1:
                idx, val, _, _ = hx.local(als_wins, self.offset)
                return idx, val
            a_mm, t_mm = hx.minmax()
        else:
            inf = float("inf")
            a_mm = torch.tensor([[inf] * B, [-inf] * B], dtype=torch.float32, device=dev)
            t_mm = a_mm.clone()
        if self.world > 1:
            a_mm, t_mm = global_minmax(a_mm, t_mm, self.group)
        if self.n_local > 0:
            idx, val = hx.topk(a_mm, t_mm, als_wins, self.offset)
        else:
            idx = torch.empty((B, 0), dtype=torch.int64, device=dev)
            val = torch.empty((B, 0), dtype=torch.float64, device=dev)
        if self.world == 1:
            return idx, val
        return merge_candidates(idx, val, top_k, self.world, self.group, o)

    def recommend(self, user_rows, user_vecs, als_wins, top_k):
        """user_rows: [B] int64 ALS rows; user_vecs: [B, d] two-tower user
        vectors. Returns (global item ids [B, k], fused scores f64 [B, k])."""
        if self.precision == "bf16" and self.pruned and 1 <= int(top_k) <= _hrec.PRUNE_MAX_K:
            return self._recommend_pruned(user_rows, user_vecs, als_wins, top_k)
        if (self.pruned_exact and 1 <= int(top_k) <= _hrec.EXACT_MAX_K and int(user_rows.shape[0]) >= 8
                and user_vecs.dtype == torch.float32 and user_vecs.stride(1) == 1):
            return self._recommend_exact_pruned(user_rows, user_vecs, als_wins, top_k)
        o = self.ops
        B = int(user_rows.shape[0])
        dev = user_vecs.device
        if self.n_local > 0 and self.precision == "bf16" and hasattr(o, "hybrid_scores"):
            # one launch: user gather + bf16 conversion, both score GEMMs and
            # both rows' min / max (hrec_hybrid_scores; same values as below)
            als, tt, a_mm, t_mm = o.hybrid_scores(self.U, user_rows, user_vecs, self.V_op, self.iv_op)
        elif self.n_local > 0:
            als, tt = self._scores(user_rows, user_vecs)
            a_mm = o.rows_minmax(als)
            t_mm = o.rows_minmax(tt)
        else:  # an empty shard contributes neutral min/max and no candidates
            inf = float("inf")
            a_mm = torch.tensor([[inf] * B, [-inf] * B], dtype=torch.float32, device=dev)
            t_mm = a_mm.clone()
        if self.world > 1:
            a_mm, t_mm = global_minmax(a_mm, t_mm, self.group)
        if self.n_local > 0:
            idx, val = o.fuse_rows_topk(als, tt, a_mm, t_mm, als_wins, top_k, self.offset)
        else:
            idx = torch.empty((B, 0), dtype=torch.int64, device=dev)
            val = torch.empty((B, 0), dtype=torch.float64, device=dev)
        if self.world == 1:
            return idx, val
        return merge_candidates(idx, val, top_k, self.world, self.group, o)


# Collective calls issued by this module (C2 + C3): two per sharded batch.
COLLECTIVE_CALLS = [0]


def global_minmax(a_mm, t_mm, group):
    """C2: both models' per-user [min; max] rows made global in ONE
    all_reduce(MIN): the maxima travel negated (-max(x) = min(-x), exact in
    floating point), packed as [a_min | t_min | -a_max | -t_max] ([4, B] f32),
    and are negated back. Returns (als_mm, tt_mm), [2, B] each."""
    pack = torch.stack([a_mm[0], t_mm[0], -a_mm[1], -t_mm[1]])
    COLLECTIVE_CALLS[0] += 1
    dist.all_reduce(pack, op=dist.ReduceOp.MIN, group=group)
    return torch.stack([pack[0], -pack[2]]), torch.stack([pack[1], -pack[3]])


def merge_candidates(idx, val, top_k, world, group, ops):
    """C3: all_gather every rank's [B, <=k] candidates (global ids, -1 = empty
    slot) and merge them by a keyed stable top-k (ties -> smaller id). Ids
    (int64) and scores (f64, bit-cast to int64) travel as ONE [B, 2k] buffer."""
    B = idx.shape[0]
    dev = idx.device
    kk = int(top_k)
    val = val.double()  # exact for f32 scores
    if idx.shape[1] < kk:  # every rank contributes k slots; -1 marks an empty one
        pad = kk - idx.shape[1]
        idx = torch.cat([idx, torch.full((B, pad), -1, dtype=torch.int64, device=dev)], 1)
        val = torch.cat([val, torch.full((B, pad), float("-inf"), dtype=val.dtype, device=dev)], 1)
    send = torch.cat([idx.to(torch.int64), val.view(torch.int64)], 1).contiguous()
    # rank-major concatenation [W*B, 2k] (the layout every backend accepts)
    got = torch.empty((world * B, 2 * kk), dtype=torch.int64, device=dev)
    COLLECTIVE_CALLS[0] += 1
    dist.all_gather_into_tensor(got, send, group=group)
    got = got.view(world, B, 2 * kk).permute(1, 0, 2)
    cand_i = got[:, :, :kk].reshape(B, world * kk).contiguous()
    cand_v = got[:, :, kk:].contiguous().view(torch.float64).reshape(B, world * kk).contiguous()
    return ops.topk_keyed(cand_v, cand_i, top_k)


class ShardedScorer:
    """Two-tower (or any dot-product) top-k over an item axis sharded across
    ranks: rank r holds item rows [offset, offset + n_local) of the candidate
    matrix as a dot operand (hrec dot_operand: f32 or bf16, width 32..256)."""

    def __init__(self, item_vecs_local, item_offset, world=1, rank=0, group=None, ops=None):
        self.iv = item_vecs_local
        self.n_local = item_vecs_local.shape[0]
        self.offset = int(item_offset)
        self.world, self.rank, self.group = int(world), int(rank), group
        self.ops = ops or DeviceOps

    def topk(self, user_vecs, top_k):
        """user_vecs: [B, width] dot operand. Returns (global item ids [B, k],
        scores [B, k]) — f32 on one rank, f64 after the merge."""
        B = user_vecs.shape[0]
        dev = user_vecs.device
        if self.n_local > 0:
            idx, val = self.ops.dot_topk(user_vecs, self.iv, top_k, self.offset)
        else:
            idx = torch.empty((B, 0), dtype=torch.int64, device=dev)
            val = torch.empty((B, 0), dtype=torch.float32, device=dev)
        if self.world == 1:
            return idx, val
        return merge_candidates(idx, val.double(), top_k, self.world, self.group, self.ops)


class CapturedRecommend:
    """One ShardedRecommender.recommend batch captured as a HIP graph and
    replayed: a serving loop with a fixed batch size launches the whole
    hybrid (operand conversion, two score GEMMs, row min/max, fusion
    threshold filter, merge) as one graph instead of ~15 kernel launches
    from Python. Every step is device-side (no host round trip: the fusion's
    overflow fallback is gated on the device), so the graph holds the exact
    eager computation. Single rank only (W > 1 runs the collectives eagerly).

        cap = CapturedRecommend(rec, user_rows, user_vecs, als_wins, top_k)
        idx, val = cap(new_user_rows, new_user_vecs)   # same shapes

    Each call returns fresh tensors (copies of the graph's static outputs, B x k
    elements), so results kept or queued by a serving loop are not overwritten
    by the next replay.
    """

    def __init__(self, rec, user_rows, user_vecs, als_wins, top_k, warmup=2):
        if rec.world != 1:
            raise ValueError("CapturedRecommend: single-rank recommenders only")
        self.rows = user_rows.clone()
        self.vecs = user_vecs.clone()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm up allocator / lazy init outside the capture
            for _ in range(warmup):
                rec.recommend(self.rows, self.vecs, als_wins, top_k)
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = rec.recommend(self.rows, self.vecs, als_wins, top_k)

    def __call__(self, user_rows=None, user_vecs=None):
        if user_rows is not None:
            self.rows.copy_(user_rows)
        if user_vecs is not None:
            self.vecs.copy_(user_vecs)
        self.graph.replay()
        return self.out[0].clone(), self.out[1].clone()
