"""Diagnostic: 2 ranks on cuda:0 over gloo running distributed.align_slabs with progress logging.

    python -u tools/dist_gpu_diag.py [m] [n] [band]
"""
import faulthandler
import os
import random
import socket
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(rank, *a):
    print(f"[{time.monotonic():.3f} r{rank}]", *a, flush=True)


def worker(rank, world, port, m, n, band):
    faulthandler.dump_traceback_later(90, exit=True)
    import torch
    import torch.distributed as dist
    from globalign_amd import distributed
    from globalign_amd._native import CostTables
    from globalign_amd.scoring import validate_and_transform_args
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s1, s2 = bench.splitmix(m, 1), bench.splitmix(n, 2)
    tables, _ = bench.problem_tables(s1, s2)
    links = distributed.Links(dist, rank, world)
    eng = distributed.GpuSlabEngine(0)
    orig_out, orig_in = eng.out_progress, eng.set_in_progress
    last = [0, time.monotonic()]

    def out_progress():
        v = orig_out()
        if v != last[0] or time.monotonic() - last[1] > 2:
            log(rank, "out_progress", v)
            last[0], last[1] = v, time.monotonic()
        return v

    def set_in(rows):
        log(rank, "set_in_progress", rows)
        orig_in(rows)

    eng.out_progress, eng.set_in_progress = out_progress, set_in
    random.seed(0)
    mt = np.array(random.getstate()[1], dtype=np.uint32)
    log(rank, "start")
    res = distributed.align_slabs(dist, links, eng, s1, s2, tables.codes(s1), tables.codes(s2), tables, mt,
                                  band=band, torch=torch)
    log(rank, "done", None if res is None else (res[0], len(res[1][0]), res[2]))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
    band = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(worker, args=(2, port, m, n, band), nprocs=2, join=True, start_method="spawn")
