"""Multi-rank path with the product engine on one MI355X: two ranks on cuda:0 over gloo.

Both ranks' slab fills run concurrently on the same GPU.  The edges cross either
through IPC-mapped device memory that each fill stores into itself (edge mode
"ipc", the default: the cross-process hand-off bench.py --gpus N uses between
GPUs), or in row bands through pinned host tensors (the gloo transport) with
progress words in pinned host memory, as distributed.py drives RCCL bands
(GA_SLAB_EDGE=bands).  The result must equal the single-problem oracle.
"""
import os
import random
import socket

import numpy as np
import pytest

from tests.conftest import splitmix_seq, set_knob, del_knob

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _parent_options():
    from globalign_amd import _native
    return dict(_native.OPTIONS)


def _scoring(seq_1, seq_2):
    from globalign_amd.scoring import validate_and_transform_args
    _, _, _, cmat, _, goc, _ = validate_and_transform_args(None, None, seq_1[:64], seq_2[:64], match_score=2,
                                                           mismatch_score=-3, gap_open_score=-5,
                                                           gap_extension_score=-1)
    return cmat, goc


def _worker(rank, world, port, seq_1, seq_2, mt_words, band, out_path, traceback=True, fail_import=False,
            fail_export=False, options=None):
    import torch
    import torch.distributed as dist
    from globalign_amd import _native, distributed
    from globalign_amd._native import CostTables
    _native.OPTIONS.update(options or {})  # the parent's context options (a spawned rank starts without them)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cmat, goc = _scoring(seq_1, seq_2)
        tables = CostTables(cmat, goc)
        links = distributed.Links(dist, rank, world)
        eng = distributed.GpuSlabEngine(0)
        if fail_import and rank == 0:
            def refuse(handle):
                raise RuntimeError("simulated: the right neighbour's IPC handle does not open")
            eng.slab_link_import = refuse
        if fail_export and rank == world - 1:
            def no_handle():
                raise RuntimeError("simulated: hipIpcGetMemHandle fails on this rank")
            eng.slab_link_export = no_handle
        for _ in range(2):  # the second run reuses the context (buffers, progress words)
            res = distributed.align_slabs(dist, links, eng, seq_1, seq_2, tables.codes(seq_1),
                                          tables.codes(seq_2), tables, mt_words, band=band, torch=torch,
                                          traceback=traceback)
        if fail_import or fail_export:
            assert links.ipc_ok is False  # every rank fell back to bands
        if rank == 0:
            cost, strings, status, mt_after = res
            if traceback:
                np.savez(out_path, cost=cost, a=strings[0], mid=strings[1], b=strings[2], status=status,
                         mt=np.asarray(mt_after, dtype=np.uint32))
            else:
                np.savez(out_path, cost=cost, status=status)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("edge", ["ipc", "bands"])
@pytest.mark.parametrize("world,m,n,seed,band", [(2, 3000, 5000, 21, 512), (3, 2100, 4100, 8, 700),
                                                  (8, 1500, 8 * 512, 31, 512)])
def test_gpu_slabs_edge_modes_match_oracle(world, m, n, seed, band, edge, tmp_path, monkeypatch):
    """World sizes 2, 3 and 8 (the driver's 8-GPU node: here 8 rank processes share the MI355X, one 512-column
    slab each, seven links, the walk handed over seven times)."""
    monkeypatch.setenv("GA_SLAB_EDGE", edge)
    _slabs_match_oracle(world, m, n, seed, band, tmp_path)


def _slabs_match_oracle(world, m, n, seed, band, tmp_path):
    import torch.multiprocessing as mp
    from oracle import core
    seq_1, seq_2 = splitmix_seq(m, seed, "dna"), splitmix_seq(n, seed + 1, "dna")
    random.seed(seed)
    mt_words = np.array(random.getstate()[1], dtype=np.uint32)
    out = str(tmp_path / "res.npz")
    mp.start_processes(_worker, args=(world, _free_port(), seq_1, seq_2, mt_words, band, out, True, False, False,
                                      _parent_options()), nprocs=world, join=True, start_method="spawn")
    r = np.load(out)
    cmat, goc = _scoring(seq_1, seq_2)
    ref = core.align(seq_1, seq_2, cmat, goc, mt_words)
    assert int(r["cost"]) == ref["cost"]
    assert (str(r["a"]), str(r["mid"]), str(r["b"])) == tuple(ref["strings"])
    assert r["mt"].tolist() == np.asarray(ref["mt_out"], dtype=np.uint32).tolist()


@pytest.mark.parametrize("edge", ["ipc", "bands"])
@pytest.mark.parametrize("world,m,n,seed,band", [(2, 4000, 60_000, 41, 1024), (3, 3000, 40_000, 43, 600)])
def test_gpu_slabs_score_only_edge_modes_match_oracle(world, m, n, seed, band, edge, tmp_path, monkeypatch):
    monkeypatch.setenv("GA_SLAB_EDGE", edge)
    _slabs_score_only_match_oracle(world, m, n, seed, band, tmp_path)


def _slabs_score_only_match_oracle(world, m, n, seed, band, tmp_path):
    """Strong-scaling bench path (C4 shape): score only, each rank's slab many workgroup slabs (60k columns
    over 2 ranks = 2 x 118 workgroups).  The ranks share one GPU here, so all their workgroups must be
    co-resident (<= 256 CUs; each rank's first slab waits on the other rank).  Cost vs the C oracle."""
    import torch.multiprocessing as mp
    from oracle import core
    from globalign_amd._native import CostTables
    seq_1, seq_2 = splitmix_seq(m, seed, "dna"), splitmix_seq(n, seed + 1, "dna")
    random.seed(seed)
    mt_words = np.array(random.getstate()[1], dtype=np.uint32)
    out = str(tmp_path / "res_so.npz")
    mp.start_processes(_worker, args=(world, _free_port(), seq_1, seq_2, mt_words, band, out, False, False, False,
                                      _parent_options()), nprocs=world, join=True, start_method="spawn")
    r = np.load(out)
    cmat, goc = _scoring(seq_1, seq_2)
    tab = core.Tables(cmat)
    a, b = tab.codes(seq_1), tab.codes(seq_2)
    big = (tab.max_cost + 1) * max(m, n)
    row0, col0 = core.boundary(tab, a, b, goc, big)
    assert int(r["cost"]) == int(min(core.fill_score_parallel(tab, a, b, goc, row0, col0, 4)))


@pytest.mark.parametrize("td", [1, 2])
def test_gpu_slabs_score_only_diag_match_oracle(td, monkeypatch, tmp_path):
    """The anti-diagonal fill (GA_FILL_MODE=diag; no longer chosen automatically) in slab mode:
    the left edge from the neighbour rank's progress word, the right edge out to it, the cost from the last
    rank."""
    set_knob(monkeypatch, "GA_FILL_MODE", "diag")
    set_knob(monkeypatch, "GA_DIAG_COLS_PER_LANE", str(td))
    _slabs_score_only_match_oracle(2, 4000, 30_000 + 77, 45 + td, 1024, tmp_path)
    _slabs_score_only_match_oracle(3, 12_000, 2_000 + 5, 47 + td, 2048, tmp_path)


@pytest.mark.parametrize("devices,m,n,seed,kw", [
    ([0, 0], 2500, 4100, 41, dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)),
    ([0, 0, 0], 1800, 3000, 42, dict(scoring_mat_name="BLOSUM62", gap_open_score=-10)),
])
def test_global_aligner_devices_in_process(devices, m, n, seed, kw):
    """GlobalAligner(devices=[...]): one context and slab per listed GPU in this process (slabs sharing the
    one MI355X here run in turn), the result bit-exact with the oracle, the random state included."""
    import globalign_amd
    from oracle import core, transform
    from tests.conftest import load_matrix
    alpha = "protein" if "scoring_mat_name" in kw else "dna"
    s1, s2 = splitmix_seq(m, seed, alpha), splitmix_seq(n, seed + 1, alpha)
    blosum = load_matrix(kw["scoring_mat_name"]) if "scoring_mat_name" in kw else None
    a1, a2, _, cmat, _, goc = transform.settings(dict(kw, seq_1=s1, seq_2=s2), blosum=blosum)
    random.seed(seed)
    ref = core.align(a1, a2, cmat, goc, core.mt_state_array())
    random.seed(seed)
    r = globalign_amd.GlobalAligner(max_seq_len_prod=None, devices=devices, **kw).align(s1, s2)
    assert r.cost == ref["cost"]
    assert (r.seq_1_aligned, r.middle_part, r.seq_2_aligned) == tuple(ref["strings"])
    assert random.getstate()[1] == tuple(int(x) for x in ref["mt_out"])
    r2 = globalign_amd.GlobalAligner(max_seq_len_prod=None, devices=devices, traceback=False, **kw).align(s1, s2)
    assert r2.cost == ref["cost"] and r2.seq_1_aligned is None


@pytest.mark.parametrize("world,m,n,seed,band", [(2, 3000, 5000, 51, 512), (3, 2100, 4100, 52, 700)])
def test_gpu_slabs_recompute_walk_match_oracle(world, m, n, seed, band, tmp_path, monkeypatch):
    """Traceback across slabs through the recompute walk: each rank's slab
    fill stores checkpoints only (no m x n words, so C4 traceback fits at N = 2 / 4), and each slab walk,
    handed on right to left, recomputes the blocks ahead of it -- the leftmost slabs' stripe 0 from the
    halo the left neighbour sent."""
    set_knob(monkeypatch, "GA_RC", "1")
    _slabs_match_oracle(world, m, n, seed, band, tmp_path)


def test_global_aligner_devices_recompute_walk(monkeypatch):
    """GlobalAligner(devices=[0, 0]) with the recompute walk on each slab."""
    set_knob(monkeypatch, "GA_RC", "1")
    test_global_aligner_devices_in_process([0, 0], 2600, 4200, 53, dict(match_score=2, mismatch_score=-3,
                                                                        gap_open_score=-5, gap_extension_score=-1))


def test_linked_slabs_abort_propagates(monkeypatch):
    """ga_slab_link's error path: of three linked slabs only the middle and right ones are launched, so the
    middle fill's wait for its left edge runs out (a short GA_HALO_SPIN_LIMIT); it marks its right edge
    aborted, and the right fill -- launched with the default ~30 s limit -- stops at once instead of
    waiting that out.  Both finishes raise; the same contexts then align a problem exactly."""
    import time
    from globalign_amd import _native, distributed
    from globalign_amd.scoring import validate_and_transform_args
    from oracle import core, transform
    kw = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)
    m, n = 3000, 6144
    s1, s2 = splitmix_seq(m, 61, "dna"), splitmix_seq(n, 62, "dna")
    _, _, _, cmat, _, goc, _ = validate_and_transform_args(None, None, s1[:64], s2[:64], **kw)
    tables = _native.CostTables(cmat, goc)
    a, b = tables.codes(s1), tables.codes(s2)
    # GA_* knobs are read when a context is created: only the middle slab's context gets the short halo bound
    engines = [distributed.GpuSlabEngine(0)]
    set_knob(monkeypatch, "GA_HALO_SPIN_LIMIT", str(1 << 16))
    engines.append(distributed.GpuSlabEngine(0))
    del_knob(monkeypatch, "GA_HALO_SPIN_LIMIT")
    engines.append(distributed.GpuSlabEngine(0))
    try:
        edges = distributed.slab_bounds(n, 3)
        for k, eng in enumerate(engines):
            eng.load_slab(a, b, tables, edges[k], edges[k + 1])
        engines[0].slab_link(engines[1])
        engines[1].slab_link(engines[2])
        engines[1].slab_launch(traceback=False)
        t0 = time.monotonic()
        engines[2].slab_launch(traceback=False)
        with pytest.raises(_native.EngineError):
            engines[1].slab_finish()
        with pytest.raises(_native.EngineError):
            engines[2].slab_finish()
        assert time.monotonic() - t0 < 10.0
        # the contexts recover: a full linked alignment on them
        a1, a2, _, cmat_o, _, goc_o = transform.settings(dict(kw, seq_1=s1, seq_2=s2))
        random.seed(5)
        ref = core.align(a1, a2, cmat_o, goc_o, core.mt_state_array())
        random.seed(5)
        mt = np.array(random.getstate()[1], dtype=np.uint32)
        cost, strings, status, mt_after = distributed.align_devices([0, 0, 0], s1, s2, a, b, tables, mt,
                                                                    engines=engines)
        assert status == 0 and cost == ref["cost"] and tuple(strings) == tuple(ref["strings"])
        assert np.asarray(mt_after, dtype=np.uint32).tolist() == [int(x) for x in ref["mt_out"]]
    finally:
        for eng in engines:
            eng.eng.close()


def test_gpu_slabs_ipc_failure_falls_back_to_bands(tmp_path):
    """If any rank cannot link its edges through IPC (here rank 0's import is made to fail), every rank agrees
    on the first problem to use bands instead, and the results stay exact."""
    import torch.multiprocessing as mp
    from oracle import core
    m, n, seed, world = 2500, 4600, 71, 3
    seq_1, seq_2 = splitmix_seq(m, seed, "dna"), splitmix_seq(n, seed + 1, "dna")
    random.seed(seed)
    mt_words = np.array(random.getstate()[1], dtype=np.uint32)
    out = str(tmp_path / "res_fb.npz")
    mp.start_processes(_worker, args=(world, _free_port(), seq_1, seq_2, mt_words, 600, out, True, True), nprocs=world,
                       join=True, start_method="spawn")
    r = np.load(out)
    cmat, goc = _scoring(seq_1, seq_2)
    ref = core.align(seq_1, seq_2, cmat, goc, mt_words)
    assert int(r["cost"]) == ref["cost"]
    assert (str(r["a"]), str(r["mid"]), str(r["b"])) == tuple(ref["strings"])
    assert r["mt"].tolist() == np.asarray(ref["mt_out"], dtype=np.uint32).tolist()


def test_gpu_slabs_ipc_export_failure_falls_back_to_bands(tmp_path):
    """the last rank's export fails; it still sends its neighbour a (None) handle, every rank agrees on
    bands at once (no wait for the process group's timeout), and the results stay exact."""
    import torch.multiprocessing as mp
    from oracle import core
    m, n, seed, world = 2400, 4500, 73, 3
    seq_1, seq_2 = splitmix_seq(m, seed, "dna"), splitmix_seq(n, seed + 1, "dna")
    random.seed(seed)
    mt_words = np.array(random.getstate()[1], dtype=np.uint32)
    out = str(tmp_path / "res_fe.npz")
    mp.start_processes(_worker, args=(world, _free_port(), seq_1, seq_2, mt_words, 600, out, True, False, True),
                       nprocs=world, join=True, start_method="spawn")
    r = np.load(out)
    cmat, goc = _scoring(seq_1, seq_2)
    ref = core.align(seq_1, seq_2, cmat, goc, mt_words)
    assert int(r["cost"]) == ref["cost"]
    assert (str(r["a"]), str(r["mid"]), str(r["b"])) == tuple(ref["strings"])
    assert r["mt"].tolist() == np.asarray(ref["mt_out"], dtype=np.uint32).tolist()
