"""Multi-rank path (globalign_amd/distributed.py) on CPU: gloo, world sizes 2 and 3.

The product's orchestration (slab split, banded edge exchange driven by the
progress words, right-to-left walk hand-off, assembly on rank 0) runs
unchanged; the engine under it is a CPU stand-in built on the oracle: a
background thread fills the slab band by band, waiting on the left-edge
progress word and publishing its right edge, exactly the protocol the GPU
fill follows.  The walk restates dp_array_backward (globaligner.py:395-593)
with the slab cut.  Rank 0's result must equal the single-problem oracle.
"""
import os
import random
import socket
import threading

import numpy as np
import pytest

from tests.conftest import splitmix_seq

SIZES = [3, 2, 2, 2, 3, 2, 2, 2, 3] * 2  # the dispatcher's draws per step (test_host_cpu.py)


def _levels(draws, am, S):
    q = draws[0:9] if am else draws[9:18]
    return {1: 0, 2: 1, 3: q[1], 4: 2, 5: 2 * q[2], 6: 1 + q[3], 7: q[0]}[S]


def _argmin_set(a, b, c):
    h = min(a, b, c)
    return (a == h) | ((b == h) << 1) | ((c == h) << 2)


class OracleSlabEngine:
    """CPU engine with distributed.py's slab interface (test infrastructure)."""

    def __init__(self, cmat, gap_open_cost):
        from oracle import core
        self.core = core
        self.tab = core.Tables(cmat)
        self.o = int(gap_open_cost)

    def load_slab(self, a_codes, b_codes, tables, c0, c1):
        core = self.core
        self.a = np.frombuffer(bytes(a_codes), dtype=np.uint8).copy()
        self.b_all = np.frombuffer(bytes(b_codes), dtype=np.uint8).copy()
        self.m, self.n_all = len(self.a), len(self.b_all)
        self.c0, self.c1 = c0, c1
        big = (self.tab.max_cost + 1) * max(self.m, self.n_all)
        self.row0, self.col0 = core.boundary(self.tab, self.a, self.b_all, self.o, big)
        self.in_prog = 0
        self.out_prog = 0

    def halo_shape(self, m):
        return (m + 1, 3)

    def halo_dtype(self):
        import torch
        return torch.int64

    def pinned_halos(self):
        return False

    def slab_bind_halos(self, in_ptr, out_ptr, halo_in=None, halo_out=None):
        self.halo_in = halo_in.numpy()
        self.halo_out = halo_out.numpy()

    def _fill(self, band):
        core, m = self.core, self.m
        nl = self.c1 - self.c0
        b = self.b_all[self.c0:self.c1].copy()
        dp = np.zeros((m + 1, nl + 1, 3), np.int64)
        dp[0] = self.row0.reshape(-1, 3)[self.c0:self.c1 + 1]
        for r0 in range(1, m + 1, band):
            r1 = min(m, r0 + band - 1)
            if self.c0 == 0:
                dp[r0:r1 + 1, 0] = self.col0.reshape(-1, 3)[r0:r1 + 1]
            else:
                while self.in_prog < r1:
                    threading.Event().wait(1e-4)
                dp[r0:r1 + 1, 0] = self.halo_in[r0:r1 + 1]
            sub = np.ascontiguousarray(dp[r0 - 1:r1 + 1])
            core.fill_full(self.tab, self.a[r0 - 1:r1].copy(), b, self.o, sub)
            dp[r0 - 1:r1 + 1] = sub
            self.halo_out[r0:r1 + 1] = dp[r0:r1 + 1, nl]
            self.out_prog = r1
        self.dp = dp

    def slab_launch(self, traceback=True):
        self.thread = threading.Thread(target=self._fill, args=(37,), daemon=True)
        self.thread.start()

    def out_progress(self):
        return self.out_prog

    def set_in_progress(self, rows):
        self.in_prog = rows

    def slab_finish(self):
        self.thread.join()
        return int(self.dp[self.m, self.c1 - self.c0].min())

    def slab_walk_prepare(self, mt_words):
        self.mt0 = np.array(mt_words, dtype=np.uint32)

    def _rng_at(self, D):
        r = random.Random()
        r.setstate((3, tuple(int(x) for x in self.mt0), None))
        for _ in range(D):
            for s in SIZES:
                r.choice(range(s))
        return r

    def slab_walk(self, state, seq_1, seq_2):
        i, j, D, h, L, first, reason = state
        o, c0, dp = self.o, self.c0, self.dp
        rng = self._rng_at(D)
        out = ([], [], [])
        while True:
            M, X, Y = (int(v) for v in dp[i, j - c0])
            S = _argmin_set(M, X, Y) if L == 0 else _argmin_set(M + o, X, Y + o) if L == 1 else \
                _argmin_set(M + o, X + o, Y)
            ca, cb = seq_1[i - 1], seq_2[j - 1]
            lv = _levels([rng.choice(range(s)) for s in SIZES], ca == cb, S)
            if lv == 0:
                col = (ca, "|" if ca == cb else "*", cb)
            elif lv == 1:
                col = ("-", " ", cb)
            else:
                col = (ca, " ", "-")
            for k in range(3):
                out[k].append(col[k])
            D += 1
            i -= lv != 1
            j -= lv != 2
            L = lv
            if first:
                first = 0
                if i == 0 and j == 0:
                    reason = 0
                    break
                continue
            if i == 0:
                reason = 1
                break
            if j == c0:
                reason = 5 if c0 > 0 else 2
                break
            h += 1
            if h >= self.m + self.n_all:
                reason = 3
                break
        return tuple("".join(x) for x in out), [i, j, D, h, L, first, reason]

    def slab_mt_state(self, D):
        return np.array(self._rng_at(D).getstate()[1], dtype=np.uint32)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _scoring(seq_1, seq_2):
    from globalign_amd.scoring import validate_and_transform_args
    _, _, _, cmat, _, goc, _ = validate_and_transform_args(None, None, seq_1[:64], seq_2[:64], match_score=2,
                                                           mismatch_score=-3, gap_open_score=-5,
                                                           gap_extension_score=-1)
    return cmat, goc


def _worker(rank, world, port, seq_1, seq_2, mt_words, band, out_path, traceback=True):
    import torch
    import torch.distributed as dist
    from globalign_amd import distributed
    from globalign_amd._native import CostTables
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cmat, goc = _scoring(seq_1, seq_2)
        tables = CostTables(cmat, goc)
        links = distributed.Links(dist, rank, world)
        eng = OracleSlabEngine(cmat, goc)
        res = distributed.align_slabs(dist, links, eng, seq_1, seq_2, tables.codes(seq_1), tables.codes(seq_2),
                                      tables, mt_words, band=band, torch=torch, traceback=traceback)
        if rank == 0:
            cost, strings, status, mt_after = res
            if traceback:
                np.savez(out_path, cost=cost, a=strings[0], mid=strings[1], b=strings[2], status=status,
                         mt=np.asarray(mt_after, dtype=np.uint32))
            else:
                assert strings is None and mt_after is None
                np.savez(out_path, cost=cost, status=status)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _run(world, m, n, seed, band, tmp_path, traceback=True):
    import torch.multiprocessing as mp
    seq_1, seq_2 = splitmix_seq(m, seed, "dna"), splitmix_seq(n, seed + 1, "dna")
    random.seed(seed)
    mt_words = np.array(random.getstate()[1], dtype=np.uint32)
    out = str(tmp_path / f"res_{world}_{seed}.npz")
    mp.start_processes(_worker, args=(world, _free_port(), seq_1, seq_2, mt_words, band, out, traceback),
                       nprocs=world, join=True, start_method="fork")
    return seq_1, seq_2, mt_words, np.load(out)


@pytest.mark.parametrize("world,m,n,seed,band", [(2, 150, 260, 11, 40), (3, 201, 333, 5, 64), (2, 97, 130, 3, 16)])
def test_slabs_match_single_problem_oracle(world, m, n, seed, band, tmp_path):
    from oracle import core
    seq_1, seq_2, mt_words, r = _run(world, m, n, seed, band, tmp_path)
    cmat, goc = _scoring(seq_1, seq_2)
    ref = core.align(seq_1, seq_2, cmat, goc, mt_words)
    assert int(r["cost"]) == ref["cost"]
    assert (str(r["a"]), str(r["mid"]), str(r["b"])) == tuple(ref["strings"])
    assert int(r["status"]) == 0
    assert r["mt"].tolist() == np.asarray(ref["mt_out"], dtype=np.uint32).tolist()


@pytest.mark.parametrize("world,m,n,seed,band", [(2, 180, 300, 7, 50), (4, 120, 420, 9, 32)])
def test_slabs_score_only_match_oracle(world, m, n, seed, band, tmp_path):
    """The strong-scaling bench path (C4): fill + score only, no walk; the cost equals the single-problem oracle."""
    from oracle import core
    seq_1, seq_2, mt_words, r = _run(world, m, n, seed, band, tmp_path, traceback=False)
    cmat, goc = _scoring(seq_1, seq_2)
    ref = core.align(seq_1, seq_2, cmat, goc, mt_words)
    assert int(r["cost"]) == ref["cost"] and int(r["status"]) == 0


def test_slab_bounds_and_bands():
    from globalign_amd.distributed import bands, slab_bounds
    e = slab_bounds(100_000, 8)
    assert e[0] == 0 and e[-1] == 100_000 and all(b > a for a, b in zip(e, e[1:]))
    assert all(x % 64 == 0 for x in e[1:-1])
    assert slab_bounds(5, 5) == [0, 1, 2, 3, 4, 5]
    with pytest.raises(ValueError):
        slab_bounds(3, 4)
    bl = bands(1000, 256)
    assert bl[0] == (1, 256) and bl[-1] == (769, 1000) and len(bl) == 4
    # short first bands, doubling up to the band height; contiguous cover of 1..m
    bl = bands(100_000, 8192)
    assert bl[0] == (1, 512) and bl[1] == (513, 1536) and bl[-1][1] == 100_000
    assert all(b[0] == a[1] + 1 for a, b in zip(bl, bl[1:])) and max(r1 - r0 + 1 for r0, r1 in bl) == 8192
    assert bands(7, 8192) == [(1, 7)]


class _LinkOnlyEngine:
    """Just the IPC link half of the slab interface: rank `bad` cannot export its edge buffer."""

    def __init__(self, rank, bad):
        self.rank, self.bad, self.imported = rank, bad, None

    def slab_link_export(self):
        if self.rank == self.bad:
            raise RuntimeError("simulated: hipIpcGetMemHandle failed")
        return bytes([self.rank]) * 64

    def slab_link_import(self, handle):
        self.imported = handle


def _link_worker(rank, world, port, bad, out_path):
    import time
    import torch.distributed as dist
    from globalign_amd import distributed
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        links = distributed.Links(dist, rank, world)
        eng = _LinkOnlyEngine(rank, bad)
        t0 = time.monotonic()
        ok = distributed.ipc_agreed(dist, links, eng)
        np.savez(out_path + f".{rank}.npz", ok=ok, dt=time.monotonic() - t0,
                 imported=eng.imported if eng.imported is not None else b"")
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bad", [(2, 1), (3, 1), (3, 2)])
def test_ipc_export_failure_reaches_the_agreement(world, bad, tmp_path):
    """a rank whose slab_link_export raises still sends its left neighbour a (None) handle, so the
    neighbour does not wait out the process group's timeout; every rank reaches the all-reduce at once and
    agrees on bands.  Ranks whose own links worked have imported their right neighbour's handle."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "link")
    mp.start_processes(_link_worker, args=(world, _free_port(), bad, out), nprocs=world, join=True, start_method="fork")
    for r in range(world):
        res = np.load(out + f".{r}.npz")
        assert not bool(res["ok"])
        assert float(res["dt"]) < 20.0
        if r < world - 1 and bad not in (r, r + 1):
            assert bytes(res["imported"]) == bytes([r + 1]) * 64
