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


def _shard(n_users, n_items, transposed, world, rank):
    from src.als_engine import shard_range
    from src.synthetic import DeviceCSR

    total = n_items if transposed else n_users
    r0, per = shard_range(total, world, rank)
    ip, ix, v = obuild.synth_csr(n_users, n_items, DENS, int(transposed), r0, per, SEED, SEED2)
    return DeviceCSR(torch.from_numpy(ip), torch.from_numpy(ix), torch.from_numpy(v), r0, per,
                     n_users if transposed else n_items)


def _worker(rank, world, port, U0, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from src.als_engine import DeviceALS

    eng = DeviceALS(N_USERS, N_ITEMS, K, REG, _shard(N_USERS, N_ITEMS, False, world, rank),
                    _shard(N_USERS, N_ITEMS, True, world, rank), world=world, rank=rank,
                    group=dist.group.WORLD, sweep=_oracle_sweep)
    eng.set_user_factors(U0)
    eng.fit(ITERS)
    q.put((rank, eng.user_factors.numpy().copy(), eng.item_factors.numpy().copy()))
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_als_matches_unsharded(world):
    rng = np.random.default_rng(0)
    U0 = rng.normal(size=(N_USERS, K)).astype(np.float32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, U0, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ucsr = obuild.synth_csr(N_USERS, N_ITEMS, DENS, 0, 0, N_USERS, SEED, SEED2)
    icsc = obuild.synth_csr(N_USERS, N_ITEMS, DENS, 1, 0, N_ITEMS, SEED, SEED2)
    U, V = oals.fit(ucsr, icsc, U0, K, REG, ITERS, sweep=obuild.half_sweep)
    for _, Ur, Vr in res:
        np.testing.assert_array_equal(Ur, U)
        np.testing.assert_array_equal(Vr, V)


def test_shard_ranges_cover_and_pad():
    from src.als_engine import shard_range

    for n in (1, 7, 100, 1000001):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            per = spans[0][1]
            assert all(s[1] == per for s in spans)
            assert per * w >= n and per == -(-n // w)  # covers [0, n); tail shards padded
            assert [s[0] for s in spans] == [r * per for r in range(w)]
