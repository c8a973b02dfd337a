"""GPU box (one GPU): the landmark-sharded BA alone, N ranks as N processes sharing cuda:0 (the
P2P exchange over IPC-mapped buffers), each rank re-solving its 2,000-landmark shard of a
config-3-per-rank window R times; prints per rank the device ms per LM iteration (the solve's
device stamps) -- run it under rocprofv3 --kernel-trace --stats for the per-kernel split of the
sharded iteration (K4c, K5, K6[, X1][, X2]) at each RSVIO_P2P_FOLD level.
  python tools/p2p_probe.py [ranks] [repeats]          # spawns the ranks itself
  RANK=r WORLD_SIZE=n MASTER_PORT=p python tools/p2p_probe.py n [repeats]
                                                       # one rank per process, started by the shell:
                                                       # the form to run under rocprofv3 (the
                                                       # profiled program is then the rank itself)"""
import os
import socket
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "rs-vio_amd")]


def worker(rank, world, port, reps):
    import numpy as np
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rsvio import synthetic as S
        from rsvio.ba import BundleAdjuster
        shard = S.ba_problem(n_lm=2000 * world).shard(rank, world)
        ba = BundleAdjuster(max_keyframes=21, max_landmarks=shard.n_lm, max_observations=shard.n_obs)
        # PROBE_CU_SPLIT=f: the BA on bench.py's CU partition (the CUs past the tracker's block
        # fraction f), so sharded and unsharded chains compare on the same CUs as the headline
        split = float(os.environ.get("PROBE_CU_SPLIT", "0"))
        cs = None
        if split > 0:
            import bench
            from rsvio._lib import CuStream
            _, cu_ba = bench.cu_partition(0, split, "block")
            cs = CuStream(0, cu_ba)
            ba.set_stream(cs.ptr)
        # PROBE_SINGLE=1: the unsharded single-rank chain (no exchange attached) on the same stream
        single = os.environ.get("PROBE_SINGLE", "0") == "1"
        if not single:
            handles = [None] * world
            dist.all_gather_object(handles, ba.p2p_export(world))
            ba.attach_p2p(world, rank, handles)
            lat = {n: ba.p2p_latency_us(200, n) for n in (4, 1600)}
            print(f"rank {rank}: exchange latency us {lat}", flush=True)
        ba.set_problem_from(shard)
        ms = []
        # PROBE_STAMPS=1 (with RSVIO_LIB = the stamps build): K5's phase stamps of the solve's last
        # iteration, block 0 -- STAMP 0 (entry), 1 (system in LDS), 2 (fail checked), 3 (solved)
        stamps = os.environ.get("PROBE_STAMPS", "0") in ("1", "2")
        panels = os.environ.get("PROBE_STAMPS", "0") == "2"
        ph = []
        if stamps:
            import ctypes as C
            from rsvio import _lib
            buf = (C.c_ulonglong * 64)()
        for k in range(reps + 3):
            r = ba.run()
            if k >= 3:
                ms.append(r.solve_ms / max(r.iterations, 1))
                if stamps:
                    _lib.load().rsvio_dbg_ba_stamps(buf, 64)
                    # PROBE_STAMPS=2: the 8-column panels' steps instead (2 = factor start, 9 /
                    # 13 / 15 / 19 / 30 / 31 around panels 0, 2, 4, 7 = last panel, 3 = solved)
                    order = [2, 9, 13, 15, 19, 30, 31, 7, 3] if panels else [0, 1, 2, 3]
                    st = [int(buf[i]) for i in order]
                    ph.append([st[i + 1] - st[i] for i in range(len(st) - 1)])  # shader clock cycles
        if stamps:
            med = np.median(np.array(ph), axis=0)
            what = ("panel 0, 0-1, 1-2, 2-3, 3-4, 4-5, 5-6 steps, back-substitution" if panels else
                    "entry->system, ->checked, ->solved")
            print(f"rank {rank}: K5 phases, cycles ({what}) "
                  f"{' '.join(f'{v:.0f}' for v in med)}", flush=True)
        mode = "single (unsharded)" if single else f"fold {os.environ.get('RSVIO_P2P_FOLD', '3')}"
        print(f"rank {rank}: {mode} cu_split {split} ll {os.environ.get('RSVIO_P2P_LL', '0')} status {r.status} it {r.iterations} "
              f"ms/iter median {float(np.median(ms)):.4f} min {min(ms):.4f}", flush=True)
        ba.close()
        if cs is not None:
            cs.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    if "RANK" in os.environ:
        worker(int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ["MASTER_PORT"]), reps)
        sys.exit(0)
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(worker, args=(world, port, reps), nprocs=world, join=True, start_method="spawn")
