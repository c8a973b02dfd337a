"""Landmark sharding of the BA on CPU: world-size-2 `gloo` process groups.

The GPU path all-reduces each rank's partial reduced camera system (S, b, cost; lambda added on
rank 0 only) and then solves redundantly.  These tests check the decomposition that exchange
relies on with the oracle: the sum over ranks of the shard systems equals the full problem's
system, the shards partition the landmarks and observations, and a redundant solve of the
reduced system gives the same camera step on every rank.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, lam, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from rsvio import synthetic as S
        full = S.ba_problem(n_kf=6, n_lm=300, kf_per_lm=4, seed=31, init_seed=32)
        shard = full.shard(rank, world)
        # every rank damps its landmark blocks (V + lambda I); the camera diagonal's lambda is
        # added by rank 0 only (ba.hip lambda_owner), so the other ranks take it back out here
        Sm, b, cost = O.ba_build_system(shard, lam)
        n = b.size
        if rank != 0:
            Sm = Sm - lam * np.eye(n)
        t = torch.from_numpy(np.concatenate([Sm.ravel(), b, [cost]]))
        dist.all_reduce(t)  # the exchange step (RCCL ncclAllReduce on the GPU path)
        S_sum, b_sum = t[: n * n].numpy().reshape(n, n), t[n * n: n * n + n].numpy()
        # redundant dense solve on every rank (K5): identical step everywhere
        dc = np.linalg.solve(S_sum, b_sum)
        steps = [torch.zeros(n, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(steps, torch.from_numpy(dc))
        counts = torch.tensor([shard.n_lm, shard.n_obs], dtype=torch.int64)
        dist.all_reduce(counts)
        if rank == 0:
            np.savez(os.path.join(out_dir, "shard.npz"), S=S_sum, b=b_sum, cost=float(t[-1]),
                     steps=np.stack([s.numpy() for s in steps]), counts=counts.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("lam", [1e-4, 10.0])
def test_sharded_system_sums_to_full(tmp_path, lam):
    from oracle import oracle as O
    from rsvio import synthetic as S
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), lam, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r = np.load(tmp_path / "shard.npz")
    full = S.ba_problem(n_kf=6, n_lm=300, kf_per_lm=4, seed=31, init_seed=32)
    Sf, bf, cf = O.ba_build_system(full, lam)
    assert np.abs(r["S"] - Sf).max() <= 1e-9 * np.abs(Sf).max()
    assert np.abs(r["b"] - bf).max() <= 1e-9 * np.abs(bf).max()
    assert abs(float(r["cost"]) - cf) <= 1e-12 * abs(cf)
    assert np.array_equal(r["steps"][0], r["steps"][1])          # same camera step on both ranks
    assert r["counts"].tolist() == [full.n_lm, full.n_obs]        # shards partition the problem


def test_shards_partition_landmarks():
    from rsvio import synthetic as S
    full = S.ba_problem(n_kf=5, n_lm=101, kf_per_lm=3, seed=4, init_seed=5)
    for world in (2, 3, 8):
        parts = [full.shard(r, world) for r in range(world)]
        assert sum(p.n_lm for p in parts) == full.n_lm
        assert sum(p.n_obs for p in parts) == full.n_obs
        pw = np.concatenate([p.p_W for p in parts])
        assert np.array_equal(pw, full.p_W)
        for p in parts:
            assert p.obs_lm.min() >= 0 and p.obs_lm.max() < p.n_lm
