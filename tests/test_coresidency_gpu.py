"""A slab fill waiting on its halo must not hold up the kernel that delivers it.

On a multi-GPU node the halo of a slab arrives from an RCCL receive kernel that
runs WHILE the slab's persistent fill occupies every CU and polls the halo's
progress word.  Two things must hold for that not to deadlock:

* co-residency: a kernel on another stream finds room beside the fill (the fill
  takes one workgroup per CU and leaves LDS / VGPRs / wave slots free);
* queue separation: no other stream's kernel sits behind the fill in the same
  in-order hardware queue (GPU_MAX_HW_QUEUES = 4 per process: with enough
  streams, queues are shared).  The engine creates its stream with the
  device's greatest priority, which HIP serves from a separate queue pool.

The test runs that situation on one MI355X: the left slab's edge is computed
first; the right slab's fill is launched and waits; then kernels are enqueued on
many torch streams created AFTER the fill's (one of them copies the halo in with
an elementwise kernel).  Every one of them must complete while the fill is still
waiting; only then is the progress word raised.  The cost must equal the oracle's.
If a kernel cannot start, the deadline releases the fill (no hang) and the test fails.
"""
import time

import pytest

from tests.conftest import splitmix_seq

pytestmark = pytest.mark.gpu


def _scoring(seq_1, seq_2):
    from globalign_amd.scoring import validate_and_transform_args
    _, _, _, cmat, _, goc, _ = validate_and_transform_args(None, None, seq_1[:64], seq_2[:64], match_score=2,
                                                           mismatch_score=-3, gap_open_score=-5,
                                                           gap_extension_score=-1)
    return cmat, goc


def _halo_copy(stream, dst, src, rows, variant, blocks=64):
    """ga_debug_halo_copy: an RCCL-shaped copy kernel.  variant 0: 256 threads, 20 KB LDS, > 256 registers
    per lane; 1: RCCL 7.2's own gfx950 send/recv kernel resources (512 threads, 37 664 B LDS, 256 VGPRs)."""
    import ctypes as C
    from globalign_amd import _native
    f = _native.load_library().ga_debug_halo_copy
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32]
    f.restype = C.c_int
    assert f(stream, dst, src, rows, blocks, variant) == 0


def run_coresidency(m=6000, n=4096, split=2048, nstreams=8, deadline_s=10.0, traceback=False, heavy=None):
    """heavy: None (the halo lands through a torch elementwise kernel) or a ga_debug_halo_copy variant."""
    """-> dict(cost, all_done_while_waiting, waited_s, fill_still_waiting, priority, kind)."""
    import torch
    from globalign_amd import _native
    seq_1, seq_2 = splitmix_seq(m, 31, "dna"), splitmix_seq(n, 32, "dna")
    cmat, goc = _scoring(seq_1, seq_2)
    tables = _native.CostTables(cmat, goc)
    a, b = tables.codes(seq_1), tables.codes(seq_2)
    dev = torch.device("cuda:0")
    edge = torch.empty((m + 1, 2), dtype=torch.int32, device=dev)
    halo = torch.empty((m + 1, 2), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    # the left slab [0, split): its right edge into `edge`
    left = _native.Engine(0)
    left.load_slab(a, b, tables, 0, split)
    left.slab_bind_halos(0, edge.data_ptr())
    left.slab_launch(traceback)
    left.slab_finish()
    # the right slab [split, n): waits on its halo
    right = _native.Engine(0)
    right.load_slab(a, b, tables, split, n)
    right.slab_bind_halos(halo.data_ptr(), 0)
    right.wait_stream(torch.cuda.current_stream().cuda_stream)
    right.slab_launch(traceback)
    time.sleep(0.05)  # the fill is resident and spinning on its progress word
    streams = [torch.cuda.Stream(device=dev) for _ in range(nstreams)]
    events, sinks = [], []
    for k, s in enumerate(streams):
        with torch.cuda.stream(s):
            if k == nstreams // 2:
                if heavy is not None:
                    _halo_copy(s.cuda_stream, halo.data_ptr(), edge.data_ptr(), m + 1, heavy)
                else:
                    torch.add(edge, 0, out=halo)  # the halo lands through an elementwise kernel
            x = torch.arange(1 << 16, device=dev, dtype=torch.int32)
            sinks.append(x * 3 + k)
            ev = torch.cuda.Event()
            ev.record(s)
            events.append(ev)
    t0 = time.monotonic()
    done = False
    while time.monotonic() - t0 < deadline_s:
        if all(e.query() for e in events):
            done = True
            break
        time.sleep(1e-3)
    waited = time.monotonic() - t0
    fill_stream = torch.cuda.ExternalStream(right.stream(), device=dev)
    still_waiting = not fill_stream.query()  # the fill kernel has not exited
    right_priority = right.stream_priority()
    right.set_in_progress(m)  # release the fill in every case (no hang)
    cost = right.slab_finish()
    torch.cuda.synchronize()
    ok_sinks = all(int(s[5].item()) == 15 + k for k, s in enumerate(sinks))
    kind = right.fill_kind()
    left.close()
    right.close()
    return dict(cost=cost, all_done_while_waiting=done and ok_sinks, waited_s=waited,
                fill_still_waiting=still_waiting, priority=right_priority, seqs=(seq_1, seq_2), kind=kind,
                halo_ok=bool(torch.equal(halo, edge)), tables=tables)


def oracle_cost(seq_1, seq_2):
    from oracle import core
    cmat, goc = _scoring(seq_1, seq_2)
    tab = core.Tables(cmat)
    a, b = tab.codes(seq_1), tab.codes(seq_2)
    big = (tab.max_cost + 1) * max(len(a), len(b))
    row0, col0 = core.boundary(tab, a, b, goc, big)
    return int(min(core.fill_score(tab, a, b, goc, row0, col0)))


@pytest.mark.parametrize("traceback", [False, True])
def test_kernel_on_later_stream_runs_beside_waiting_slab_fill(traceback):
    r = run_coresidency(traceback=traceback)
    assert r["all_done_while_waiting"], f"kernels on later streams did not run beside the waiting fill ({r})"
    assert r["fill_still_waiting"], "the slab fill finished before its halo was released"
    assert r["cost"] == oracle_cost(*r["seqs"])


@pytest.mark.parametrize("variant", [0, 1])
def test_rccl_shaped_kernel_runs_beside_c4_slab_fill(variant):
    """The same at the geometry of a C4 slab at N = 2 (1M rows, 499 712 columns).  The halo
    arrives through a kernel shaped like RCCL's (variant 0: 256 threads, 20 KB LDS, > 256 registers per
    lane; 1: RCCL 7.2's own send/recv kernel resources, a CU of its own), which must start and finish while
    the fill waits.  A slab whose edges a kernel moves keeps one CU of every shader engine free
    (lane_geometry): here one round of at most 224 workgroups.  The cost must equal the one-GPU fill's."""
    from globalign_amd import _native
    m, split, width = 1_000_000, 2048, 499_712
    r = run_coresidency(m=m, n=split + width, split=split, heavy=variant, deadline_s=20.0)
    kind = r["kind"]
    assert kind[0] == "lane" and kind[4] <= 224, kind
    assert r["all_done_while_waiting"], f"the RCCL-shaped kernel did not run beside the waiting fill ({r})"
    assert r["fill_still_waiting"], "the slab fill finished before its halo was released"
    assert r["halo_ok"]
    eng = _native.Engine(0)
    try:
        seq_1, seq_2 = r["seqs"]
        eng.load(r["tables"].codes(seq_1), r["tables"].codes(seq_2), r["tables"])
        cost, _ = eng.fill(traceback=False)
    finally:
        eng.close()
    assert r["cost"] == cost
