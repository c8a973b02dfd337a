"""The sharded BA's attach agreement (rsvio.ba.attach_agreed) on CPU: two
`gloo` ranks drive a stand-in handle that records its calls, with a fault injected on ONE rank.
Every rank must take the same branch -- all on P2P, all detached onto RCCL, or all raising
RuntimeError when no RCCL communicator was attached -- and none may wait for a peer that left
(the solve every rank must agree on is sliding_window.rs:325's, split over landmark shards)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


class FakeHandle:
    """BundleAdjuster's attach surface: export / attach / detach / RCCL, with injectable faults."""

    def __init__(self, rank, fail_export=False, fail_attach=False):
        self.rank, self.fail_export, self.fail_attach = rank, fail_export, fail_attach
        self.calls = []
        self.collective = "none"

    def rccl_unique_id(self):
        return b"uid"

    def attach_comm(self, world, rank, uid):
        self.calls.append("comm")
        self.collective = "rccl"

    def p2p_export(self, world):
        self.calls.append("export")
        if self.fail_export:
            raise RuntimeError("injected export failure")
        return bytes([self.rank]) * 64

    def attach_p2p(self, world, rank, handles):
        self.calls.append("attach")
        assert len(handles) == world and all(len(h) == 64 for h in handles)
        if self.fail_attach:
            raise RuntimeError("injected attach failure")
        self.prev, self.collective = self.collective, "p2p"

    def detach_p2p(self):
        self.calls.append("detach")
        self.collective = self.prev


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, case, rccl_ok, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rsvio.ba import attach_agreed
        h = FakeHandle(rank, fail_export=(case == "export" and rank == 1),
                       fail_attach=(case == "attach" and rank == 0))
        try:
            got = attach_agreed(h, world, rank, "auto", rccl_ok)
        except RuntimeError:
            got = "error"
        np.save(os.path.join(out_dir, f"r{rank}.npy"),
                np.array([got, h.collective, ",".join(h.calls)], dtype=object), allow_pickle=True)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,rccl_ok,want", [
    ("none", True, "p2p"), ("none", False, "p2p"),
    ("export", True, "rccl"), ("export", False, "error"),
    ("attach", True, "rccl"), ("attach", False, "error"),
])
def test_ranks_take_the_same_branch(tmp_path, case, rccl_ok, want):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), case, rccl_ok, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    outs = [np.load(tmp_path / f"r{r}.npy", allow_pickle=True) for r in range(world)]
    assert [o[0] for o in outs] == [want] * world
    for r, (got, coll, calls) in enumerate(outs):
        calls = calls.split(",")
        assert coll == ("p2p" if want == "p2p" else "rccl" if rccl_ok else "none"), (r, coll)
        assert ("comm" in calls) == rccl_ok
        if case == "export":          # one rank had nothing to share: no rank tries to attach
            assert "attach" not in calls
        if case == "attach":          # rank 0 failed its attach: rank 1 attached, then detached
            assert ("detach" in calls) == (r == 1)
