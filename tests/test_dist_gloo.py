"""World-size-2 `gloo` test of the multi-rank reduction of the hot path (CPU only).

The only cross-rank exchange is dist.feature_mean's fused all-reduce of [sum phi, count].
Two ranks each hold a shard of the rollout's RFF features (computed with the oracle's
torch-CPU get_rep); the witness they derive must equal the single-process
fit_cost witness, and the threshold MAX-reduce must equal the global max.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from amp_extensions_amd import dist as D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        from oracle import milo_ref as R
        rs = np.random.RandomState(0)
        expert = torch.from_numpy(rs.randn(256, 20)).float()
        cost = R.RBFLinearCostRef(expert, feature_dim=128, bw_samples=2000, lambda_b=0.1, seed=3)
        x = torch.from_numpy(np.random.RandomState(1).randn(1000, 20)).float()
        lo, hi = D.shard(x.shape[0], rank, world)
        phi = cost.get_rep(x[lo:hi]).double()
        mean = D.feature_mean(phi.sum(0), float(hi - lo))
        w = mean.float() - cost.phi_e
        thr = torch.tensor([float(rank + 1) * 0.5], dtype=torch.float64)
        D.allreduce_max(thr)
        q.put((rank, w.numpy(), float(thr.item()), (lo, hi)))
    finally:
        dist.destroy_process_group()


def test_sharded_feature_mean_matches_single_process():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle import milo_ref as R
    rs = np.random.RandomState(0)
    expert = torch.from_numpy(rs.randn(256, 20)).float()
    cost = R.RBFLinearCostRef(expert, feature_dim=128, bw_samples=2000, lambda_b=0.1, seed=3)
    x = torch.from_numpy(np.random.RandomState(1).randn(1000, 20)).float()
    w_ref = (cost.get_rep(x).double().mean(0).float() - cost.phi_e).numpy()
    for rank, w, thr, (lo, hi) in res:
        np.testing.assert_allclose(w, w_ref, rtol=0, atol=1e-7)
        assert thr == 1.0
    np.testing.assert_array_equal(res[0][1], res[1][1])  # every rank holds the same witness
    assert res[0][3] == (0, 500) and res[1][3] == (500, 1000)


def test_shard_covers_range():
    for total in (1, 7, 4096, 40000):
        for world in (1, 2, 3, 8):
            spans = [D.shard(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))


def test_rank_seeds_distinct():
    assert len({D.rank_seed(7, r) for r in range(8)}) == 8
