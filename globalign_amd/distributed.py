"""Multi-GPU alignment: column slabs, banded edge exchange, walk hand-off.

One process per GPU (``torch.distributed``; backend ``nccl`` = RCCL over xGMI on
ROCm).  seq_2's columns are cut into contiguous slabs, one per rank.  Every
rank runs its slab's fill as ONE kernel launch; the wavefront crosses a slab
boundary through a single column of (H', h1') pairs.  By default (edge_mode
"ipc") rank r+1 allocates that column and a progress word in uncached memory
on its GPU and hands rank r a HIP IPC handle to it; rank r's fill stores the
rows and raises the word itself, over xGMI, while rank r+1's fill polls it --
no host thread, no RCCL kernel that would need room beside the fills
(link_ipc).  With GA_SLAB_EDGE=bands (and for CPU engines) the
column is streamed in row bands through the process group instead:

* rank r's fill publishes its right edge row by row into ``halo_out`` and a
  progress word in pinned host memory; the host thread sends each band to
  rank r+1 (``isend``) as soon as the word covers it;
* rank r+1 posts one ``irecv`` per band into ``halo_in`` and, when a band has
  landed, raises its own progress word, which the running fill polls.

No device queue ever blocks on a flag (a stream-wait packet could stall an
RCCL stream sharing its hardware queue), and the only data-path exchange is
that edge (8 B per row per slab boundary).  Each neighbouring pair gets its
own 2-rank group so the send and receive directions progress independently.

The traceback walk then runs right to left: the rank owning column n walks
its slab, hands (i, L, D, h) to its left neighbour, and so on; rank 0
assembles the columns, appends the reference's tails and reverses
(dp_array_backward, globaligner.py:395-593, cut at slab edges).

The orchestration only needs an engine exposing the slab interface of
``_native.Engine`` (load_slab, halo_shape/halo_dtype, slab_bind_halos,
slab_launch, out_progress, set_in_progress, slab_finish, slab_walk_prepare,
slab_walk, slab_mt_state); the multi-process CPU tests drive it with a CPU
engine built on the oracle.
"""
import math
import os
import threading
import time

import numpy as np

# a progress word's value once its writer gave up (ga_sync.h PROG_ABORT)
PROG_ABORT = 0xFFFFFFFF


def slab_bounds(n, world, align=512):
    """Contiguous column slabs [c_k, c_{k+1}); inner edges on multiples of `align` when n allows (512: an
    inner slab ends on a whole stripe of either fill kernel at any stripe width)."""
    if world < 1 or n < world:
        raise ValueError(f"cannot split {n} columns over {world} ranks")
    edges = [0]
    for k in range(1, world):
        e = int(round(n * k / world / align)) * align
        e = min(max(e, edges[-1] + 1), n - (world - k))
        edges.append(e)
    edges.append(n)
    return edges


def bands(m, band, first=512):
    """Row bands (r0, r1), 1-based inclusive, covering rows 1..m: `first` rows, then doubling up to `band`.

    The next rank's fill starts when the first band arrives, so the first bands are short (the
    pipeline's start-up per slab boundary: one short band instead of one `band`-row band)."""
    out, r0, h = [], 1, max(1, min(first, band))
    while r0 <= m:
        out.append((r0, min(m, r0 + h - 1)))
        r0 += h
        h = min(2 * h, band)
    return out


class Links:
    """Process groups of one rank: the pair groups with its neighbours plus a CPU control group."""

    def __init__(self, dist, rank, world):
        self.rank, self.world = rank, world
        self.left = self.right = None
        for k in range(world - 1):
            g = dist.new_group([k, k + 1])  # every rank takes part in every new_group call
            if k == rank - 1:
                self.left = g
            if k == rank:
                self.right = g
        backend = dist.get_backend()
        self.ctrl = dist.new_group(backend="gloo") if backend != "gloo" else None
        self.device_tensors = backend != "gloo"
        self.ipc_ok = None  # edge links through IPC: agreed by every rank on the first problem (ipc_agreed)
        self.ipc_linked_now = False
        self.ipc_error = None  # this rank's reason when its link failed

    def warm_up(self, dist, torch, device):
        """Create the pair communicators now (one tiny exchange each way on every pair group).

        RCCL sets a communicator up on its first send/recv; doing that while a slab fill is
        already running would put its allocations and set-up kernels beside a persistent kernel
        waiting on the very exchange being set up.  Collective over all ranks."""
        if not self.device_tensors:
            return
        buf = torch.zeros(2, dtype=torch.int32, device=device)
        for k in range(self.world - 1):
            if self.rank not in (k, k + 1):
                continue
            g = self.right if self.rank == k else self.left
            peer = k + 1 if self.rank == k else k
            for sender in (k, k + 1):
                if self.rank == sender:
                    dist.send(buf, dst=peer, group=g)
                else:
                    dist.recv(buf, src=peer, group=g)
        torch.cuda.synchronize(device)


def stream_edges(dist, links, engine, halo_in, halo_out, m, band, timeout_s=600.0, poll_s=20e-6):
    """Exchange this rank's slab edges with its neighbours while its fill runs."""
    rank, world = links.rank, links.world
    bl = bands(m, band)
    errors = []

    def receiver(recvs):
        # gloo's p2p work completes only in wait(); an NCCL work's wait() just orders streams,
        # so poll its device event instead.  Raise the progress word band by band.
        try:
            for k, w in enumerate(recvs):
                if links.device_tensors:
                    t0 = time.monotonic()
                    while not w.is_completed():
                        if time.monotonic() - t0 > timeout_s:
                            raise TimeoutError(f"rank {rank}: band {k} never arrived")
                        time.sleep(poll_s)
                else:
                    w.wait()
                engine.set_in_progress(bl[k][1])
        except Exception as e:  # surfaced by the caller
            errors.append(e)
            try:
                engine.set_in_progress(PROG_ABORT)  # the local fill stops waiting for the edge
            except Exception:
                pass

    th = None
    if rank > 0:
        recvs = [dist.irecv(halo_in[r0:r1 + 1], src=rank - 1, group=links.left) for (r0, r1) in bl]
        th = threading.Thread(target=receiver, args=(recvs,), daemon=True)
        th.start()
    sends = []
    if rank < world - 1:
        t0 = time.monotonic()
        nsent = 0
        while nsent < len(bl):
            prog = engine.out_progress()
            moved = False
            while nsent < len(bl) and prog >= bl[nsent][1]:
                r0, r1 = bl[nsent]
                sends.append(dist.isend(halo_out[r0:r1 + 1], dst=rank + 1, group=links.right))
                nsent += 1
                moved = True
            if errors:
                break
            if not moved:
                if time.monotonic() - t0 > timeout_s:
                    raise TimeoutError(f"rank {rank}: right edge stalled at {prog} rows ({nsent}/{len(bl)} bands sent)")
                time.sleep(poll_s)
    if th is not None:
        th.join()
    if errors:
        raise errors[0]
    # the sends must have READ halo_out before the next fill rewrites it: gloo completes them in
    # wait(); an NCCL work's wait() only orders streams, so poll its completion event
    t0 = time.monotonic()
    for k, w in enumerate(sends):
        if links.device_tensors:
            while not w.is_completed():
                if time.monotonic() - t0 > timeout_s:
                    raise TimeoutError(f"rank {rank}: send of band {k} never completed")
                time.sleep(poll_s)
        else:
            w.wait()


def _halos(engine, links, m, torch):
    """The slab's halo buffers, kept on the engine across steps (one allocation per problem size).

    Their contents need no reset: the fill reads halo_in only below its progress word, and the
    host sends halo_out rows only below the fill's.  With RCCL they are device tensors; with gloo
    pinned (or, for CPU engines, plain) host tensors."""
    shape, dtype = engine.halo_shape(m), engine.halo_dtype()
    key = (shape, str(dtype), links.device_tensors)
    cached = getattr(engine, "_halo_cache", None)
    if cached is not None and cached[0] == key:
        return cached[1], cached[2]
    if links.device_tensors:
        halo_in = torch.empty(shape, dtype=dtype, device=engine.torch_device())
        halo_out = torch.empty(shape, dtype=dtype, device=engine.torch_device())
    else:
        pin = engine.pinned_halos()
        halo_in = torch.zeros(shape, dtype=dtype, pin_memory=pin)
        halo_out = torch.zeros(shape, dtype=dtype, pin_memory=pin)
    engine._halo_cache = (key, halo_in, halo_out)
    return halo_in, halo_out


def edge_mode(engine):
    """How a slab's edges cross to the next rank: "ipc" -- the left fill stores them into the right rank's
    GPU memory, mapped through a HIP IPC handle (engines with slab_link_export; the default) -- or "bands"
    -- halo bands sent by the host over the process group (RCCL / gloo; GA_SLAB_EDGE=bands, CPU engines)."""
    mode = os.environ.get("GA_SLAB_EDGE", "ipc")
    if mode not in ("ipc", "bands"):
        raise ValueError(f"GA_SLAB_EDGE={mode!r}: expected 'ipc' or 'bands'")
    return mode if hasattr(engine, "slab_link_export") else "bands"


def ipc_agreed(dist, links, engine):
    """Whether every rank could link its edges through IPC, decided once per process group (the first
    problem): each rank links (`link_ipc`) and reports; if any failed -- a handle that does not open, no
    peer path between two GPUs -- every rank uses bands from then on.  Collective over all ranks."""
    if links.ipc_ok is None:
        import torch
        ok = 1
        try:
            link_ipc(dist, links, engine)
        except Exception as e:  # noqa: BLE001 (any failure to link falls back, reported on stderr)
            import sys
            print(f"rank {links.rank}: IPC edge link failed ({e}); using bands", file=sys.stderr, flush=True)
            links.ipc_error = f"{type(e).__name__}: {e}"
            ok = 0
        flag = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=links.ctrl)
        links.ipc_ok = bool(int(flag[0]))
        links.ipc_linked_now = links.ipc_ok  # this problem is already linked
    return links.ipc_ok


def edge_preflight(dist, links, engine, a_codes, b_codes, tables):
    """bench.py --gpus N, before any timed step: load this rank's slab and link its edges (ipc_agreed: every rank
    tries its IPC links, and a failure on any makes all of them use bands), then report, for each slab boundary,
    which GPUs it joins and which transport carries its edge -- so that a fallback is visible in the bench line,
    not only on stderr.  Collective over all ranks."""
    rank, world = links.rank, links.world
    edges = slab_bounds(len(b_codes), world)
    engine.load_slab(a_codes, b_codes, tables, edges[rank], edges[rank + 1])
    requested = edge_mode(engine)
    ipc = requested == "ipc" and ipc_agreed(dist, links, engine)
    dev = getattr(engine, "device", None)
    pci = None
    if dev is not None:
        try:
            import torch
            pr = torch.cuda.get_device_properties(dev)
            pci = "%04x:%02x:%02x" % (getattr(pr, "pci_domain_id", 0), getattr(pr, "pci_bus_id", 0),
                                      getattr(pr, "pci_device_id", 0))
        except Exception:  # noqa: BLE001 (diagnostic only)
            pci = None
    # every step loads its slab again (ga_problem_set_slab drops a context's links): the first step links anew
    links.ipc_linked_now = False
    info = {"rank": rank, "device": dev, "pci": pci, "ipc_error": links.ipc_error}
    everyone = [None] * world
    dist.all_gather_object(everyone, info, group=links.ctrl)
    bounds = []
    for k in range(world - 1):
        a, b = everyone[k], everyone[k + 1]
        bounds.append({"ranks": [k, k + 1], "devices": [a["device"], b["device"]], "pci": [a["pci"], b["pci"]],
                       "same_gpu": a["pci"] is not None and a["pci"] == b["pci"],
                       "transport": "ipc (the left fill stores into the right GPU's memory)" if ipc else
                       "bands (host-relayed halo bands over the process group)"})
    return {"requested": requested, "ipc_agreed": bool(ipc),
            "ipc_errors": {e["rank"]: e["ipc_error"] for e in everyone if e["ipc_error"]}, "boundaries": bounds}


def link_ipc(dist, links, engine):
    """Link this rank's slab to its neighbours for one problem: export its left-edge buffer to rank - 1, map
    rank + 1's as its right edge.  The exporter zeroes its progress word before sending the handle, and the
    importer launches its fill only after receiving it, so a fill never writes an edge its reader is still
    reading from the previous problem (that reader exports only when it starts the next)."""
    rank, world = links.rank, links.world
    err = None
    if rank > 0:
        # a failed export still sends (None): rank - 1 must not wait for a handle that never comes
        try:
            handle = engine.slab_link_export()
        except Exception as e:  # noqa: BLE001 (re-raised below, after the matching send)
            handle, err = None, e
        _send_obj(dist, handle, rank - 1, links.ctrl)
    if rank < world - 1:
        handle = _recv_obj(dist, rank + 1, links.ctrl)
        if handle is None:
            err = err or RuntimeError(f"rank {rank + 1} could not export its edge buffer")
        elif err is None:
            engine.slab_link_import(handle)
    if err is not None:
        raise err


def _send_obj(dist, obj, dst, group):
    dist.send_object_list([obj], dst=dst, group=group)


def _recv_obj(dist, src, group):
    box = [None]
    dist.recv_object_list(box, src=src, group=group)
    return box[0]


def align_slabs(dist, links, engine, seq_1, seq_2, a_codes, b_codes, tables, mt_words, band=4096, torch=None,
                traceback=True):
    """Distributed fill + traceback of one problem.  Collective over all ranks.

    Returns (cost, (seq_1_aligned, middle, seq_2_aligned), status, mt_words_after) on rank 0, None elsewhere.
    status: 0 ok, 1 the reference's IndexError.  With traceback=False only the fill runs and rank 0
    returns (cost, None, 0, None) (dp_array_forward + min of the last cell, globaligner.py:366-425)."""
    rank, world = links.rank, links.world
    m, n = len(a_codes), len(b_codes)
    edges = slab_bounds(n, world)
    c0, c1 = edges[rank], edges[rank + 1]
    engine.load_slab(a_codes, b_codes, tables, c0, c1)
    if edge_mode(engine) == "ipc" and ipc_agreed(dist, links, engine):
        # the fills store the edges into their right neighbours' memory themselves
        if links.ipc_linked_now:
            links.ipc_linked_now = False
        else:
            link_ipc(dist, links, engine)
        engine.slab_launch(traceback=traceback)
        if traceback:
            engine.slab_walk_prepare(mt_words)  # host tie-break table, overlapped with the fill
        cost = engine.slab_finish()
    else:
        halo_in, halo_out = _halos(engine, links, m, torch)
        engine.slab_bind_halos(halo_in.data_ptr() if rank > 0 else 0, halo_out.data_ptr() if rank < world - 1 else 0,
                               halo_in, halo_out)
        if links.device_tensors:
            # the halo tensors come from torch's allocator on torch's stream: the fill's stream
            # starts after whatever that stream still has in flight
            engine.order_after(torch.cuda.current_stream().cuda_stream)
        engine.slab_launch(traceback=traceback)
        if traceback:
            engine.slab_walk_prepare(mt_words)  # host tie-break table, overlapped with the fill
        stream_edges(dist, links, engine, halo_in, halo_out, m, band)
        cost = engine.slab_finish()
    ctrl = links.ctrl
    if not traceback:
        if world > 1:
            if rank == world - 1:
                _send_obj(dist, cost, 0, ctrl)
            elif rank == 0:
                cost = _recv_obj(dist, world - 1, ctrl)
        return (cost, None, 0, None) if rank == 0 else None
    # ---- walk, right to left
    if rank == world - 1:
        state = [m, n, 0, 0, 0, 1, -1]
    else:
        state = _recv_obj(dist, rank + 1, ctrl)
    seg = ("", "", "")
    if state[6] in (-1, 5):
        seg, state = engine.slab_walk(state, seq_1, seq_2)
    if rank > 0:
        _send_obj(dist, state, rank - 1, ctrl)
    # ---- assemble on rank 0
    if world > 1:
        if rank == world - 1:
            _send_obj(dist, cost, 0, ctrl)
        elif rank == 0:
            cost = _recv_obj(dist, world - 1, ctrl)
    segs = [None] * world if rank == 0 else None
    dist.gather_object(seg, segs, dst=0, group=ctrl)
    if rank != 0:
        return None
    return assemble(segs, state, cost, engine, seq_1, seq_2)


def assemble(segs, state, cost, engine, seq_1, seq_2):
    """The whole alignment from the slabs' walk segments (segs[k]: slab k's columns in walk order) and
    the final walk state: concatenate right to left, append the reference's tails, reverse
    (dp_array_backward's end, globaligner.py:542-593).  -> (cost, strings, status, mt_words_after)."""
    i, j, D, reason = state[0], state[1], state[2], state[6]
    mt_after = engine.slab_mt_state(D)
    if reason == 4:
        return cost, ("", "", ""), 1, mt_after
    sa = "".join(s[0] for s in reversed(segs))
    sm = "".join(s[1] for s in reversed(segs))
    sb = "".join(s[2] for s in reversed(segs))
    if reason == 1:  # walk hit row 0: the rest of seq_2 against gaps
        sa, sm, sb = sa + "-" * j, sm + " " * j, sb + seq_2[:j][::-1]
    elif reason == 2:  # walk hit column 0: the rest of seq_1 against gaps
        sa, sm, sb = sa + seq_1[:i][::-1], sm + " " * i, sb + "-" * i
    return cost, (sa[::-1], sm[::-1], sb[::-1]), 0, mt_after


_device_engines = {}
_device_engines_lock = threading.Lock()


def device_engines(devices):
    """The slab engines of GlobalAligner(devices=...), one context per listed device, kept for the process
    (per thread: contexts are not thread-safe) so repeated calls reuse their buffers and linked halos."""
    from globalign_amd import _native
    key = (tuple(devices), threading.get_ident(), _native.knob_fingerprint())
    with _device_engines_lock:
        engines = _device_engines.get(key)
        if engines is None:
            _native.evict_stale(_device_engines, key)
            engines = [GpuSlabEngine(d) for d in devices]
            _device_engines[key] = engines
        return engines


def align_devices(devices, seq_1, seq_2, a_codes, b_codes, tables, mt_words, traceback=True, engines=None):
    """One problem over several GPUs of THIS process (GlobalAligner(devices=[...])): one context and one
    column slab per device.  Neighbouring slabs are linked device to device (ga_slab_link): each slab's
    left edge and its progress word live in uncached memory on its own GPU, and the left neighbour's
    fill writes them directly, over xGMI, with system-scope stores while the reading fill polls the word
    (DESIGN.md 7).  No host thread relays anything; a fill that gives up marks its edge aborted, so its
    right neighbours stop too.  -> (cost, strings or None, status, mt_words_after or None)."""
    world = len(devices)
    m, n = len(a_codes), len(b_codes)
    edges = slab_bounds(n, world)
    if engines is None:
        engines = device_engines(devices)
    for k, eng in enumerate(engines):
        eng.load_slab(a_codes, b_codes, tables, edges[k], edges[k + 1])
    for k in range(world - 1):
        engines[k].slab_link(engines[k + 1])
    # left to right: a slab only ever waits on slabs launched before it (slabs sharing a GPU run in turn)
    launched, costs, error = [], [], None
    try:
        for eng in engines:
            eng.slab_launch(traceback=traceback)
            launched.append(eng)
        if traceback:
            engines[-1].slab_walk_prepare(mt_words)  # the host tie-break table, while the fills run
    except Exception as e:
        error = e
    # every launched fill is waited for, failed or not: a running fill writes into its right neighbour's
    # context, which must outlive it
    for eng in launched:
        try:
            costs.append(eng.slab_finish())
        except Exception as e:
            error = error or e
    if error is not None:
        raise error
    cost = costs[-1]
    if not traceback:
        return cost, None, 0, None
    for eng in engines[:-1]:
        eng.slab_walk_prepare(mt_words)
    state, segs = [m, n, 0, 0, 0, 1, -1], [("", "", "")] * world
    for k in range(world - 1, -1, -1):
        if state[6] in (-1, 5):
            segs[k], state = engines[k].slab_walk(state, seq_1, seq_2)
    return assemble(segs, state, cost, engines[0], seq_1, seq_2)


class GpuSlabEngine:
    """The product engine (_native.Engine) with the slab interface distributed.py drives."""

    def __init__(self, device):
        from globalign_amd import _native
        self.eng = _native.Engine(device)
        self.device = device

    def load_slab(self, a_codes, b_codes, tables, c0, c1):
        self.eng.load_slab(a_codes, b_codes, tables, c0, c1)

    def halo_shape(self, m):
        return (m + 1, 2)

    def halo_dtype(self):
        import torch
        return torch.int32

    def torch_device(self):
        return f"cuda:{self.device}"

    def pinned_halos(self):
        return True

    def slab_bind_halos(self, in_ptr, out_ptr, halo_in=None, halo_out=None):
        self.eng.slab_bind_halos(in_ptr, out_ptr)

    def slab_link(self, right):
        self.eng.slab_link(right.eng)

    def slab_link_export(self):
        return self.eng.slab_link_export()

    def slab_link_import(self, handle):
        self.eng.slab_link_import(handle)

    def order_after(self, stream):
        self.eng.wait_stream(stream)

    def slab_launch(self, traceback=True):
        self.eng.slab_launch(traceback)

    def out_progress(self):
        return self.eng.out_progress()

    def set_in_progress(self, rows):
        self.eng.set_in_progress(rows)

    def slab_finish(self):
        return self.eng.slab_finish()

    def slab_walk_prepare(self, mt_words):
        self.eng.slab_walk_prepare(mt_words)

    def slab_walk(self, state, seq_1, seq_2):
        return self.eng.slab_walk(state, seq_1, seq_2)

    def slab_mt_state(self, D):
        return self.eng.slab_mt_state(D)

    def timings(self):
        return self.eng.timings()

    def synchronize(self):
        import torch
        torch.cuda.synchronize(self.device)


def init_process_group():
    """torch.distributed from the torchrun environment (127.0.0.1 rendezvous)."""
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    backend = os.environ.get("GA_DIST_BACKEND", "nccl")
    if backend == "nccl":
        torch.cuda.set_device(local)
    dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return dist, rank, world, local


def _bench_engine(tables, local):
    """The product engine on this rank's GPU, or (GA_BENCH_ENGINE=module:factory, CPU rehearsals
    of the launcher in tests/) an engine the factory builds from the cost tables."""
    spec = os.environ.get("GA_BENCH_ENGINE")
    if spec:
        import importlib
        mod, fn = spec.split(":")
        return getattr(importlib.import_module(mod), fn)(tables)
    import torch
    return GpuSlabEngine(local % max(1, torch.cuda.device_count()))  # ranks may share a GPU (gloo rehearsal)


def bench_main(args, wl, workload):
    """bench.py --gpus N (N > 1): strong scaling of a workload over N GPUs.

    The SAME pair as the 1-GPU run (BASELINE C4 is the 1/2/4/8-GPU curve) is cut into N column
    slabs; a step is the distributed fill (+ traceback for traceback workloads) of that pair."""
    import random

    import torch

    import bench
    dist, rank, world, local = init_process_group()
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus}: torch.distributed reports {world} ranks")
    links = Links(dist, rank, world)
    m, n = wl["m"], wl["n"]
    s1, s2 = bench.workload_pair(wl)
    tables, _ = bench.problem_tables(s1, s2, wl["scoring"])
    a_codes, b_codes = tables.codes(s1), tables.codes(s2)
    random.seed(0)
    mt0 = np.array(random.getstate()[1], dtype=np.uint32)
    engine = _bench_engine(tables, local)
    # the edge links, opened and reported before timing (a fallback to bands shows in the line)
    preflight = edge_preflight(dist, links, engine, a_codes, b_codes, tables)
    if links.device_tensors:
        links.warm_up(dist, torch, engine.torch_device())
    result = None
    band = 4096 if m <= 200_000 else 8192
    fill_ms = []

    def step():
        r = align_slabs(dist, links, engine, s1, s2, a_codes, b_codes, tables, mt0, band=band, torch=torch,
                        traceback=wl["traceback"])
        fill_ms.append(engine.timings()["fill_ms"])
        return r

    for _ in range(args.warmup):
        result = step()
    fill_ms.clear()
    dist.barrier()
    engine.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        result = step()
    engine.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    stats = torch.tensor([elapsed, float(np.mean(fill_ms)) if fill_ms else 0.0], dtype=torch.float64)
    dist.all_reduce(stats, op=dist.ReduceOp.MAX, group=links.ctrl)
    elapsed, fill_max = float(stats[0]), float(stats[1])
    if rank == 0:
        cost = result[0]
        if wl["traceback"]:
            _, (sa, _, sb), status, _ = result
            assert status == 0 and sa.replace("-", "") == s1 and sb.replace("-", "") == s2
        gold = bench.golden_cost(workload)
        cells = m * n
        edges = slab_bounds(n, world)
        line = {
            "metric": bench.METRIC,
            "value": cells * args.steps / elapsed,
            "unit": "cells/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (SplitMix64, SURVEY 8d)",
            "config": {"workload": f"{wl['desc']}; {world} column slabs, "
                                   + ("edges stored by each fill into the next GPU's memory (IPC-mapped, xGMI)"
                                      if preflight["ipc_agreed"] else f"banded RCCL edge exchange ({band}-row bands)")
                                   + ("; right-to-left walk hand-off" if wl["traceback"] else ""),
                       "m": m, "n": n, "traceback": wl["traceback"], "parallelism": f"column slabs x{world}",
                       "backend": dist.get_backend(), "cost": int(cost), "oracle_cost": gold,
                       "cost_matches_oracle": (int(cost) == gold) if gold is not None else None,
                       "edge_links": preflight},
            # every rank's slab fill is one persistent launch; its time (HIP events, max over ranks)
            # includes the pipeline wait for the left neighbour's first band
            "slab_fill_ms_max": fill_max,
            "slab_columns": [b - a for a, b in zip(edges, edges[1:])],
            # the widest slab's fill against the VALU-issue bound, its instructions (and PMC bytes) per
            # cell taken from the 1-GPU launch's profile (the slab's stripe width differs: an estimate)
            "roofline": dict(bench.roofline(workload, dict(wl, n=max(b - a for a, b in zip(edges, edges[1:]))),
                                            fill_max, profile_cells=m * n),
                             note="per-cell SQ_INSTS_VALU / PMC bytes of the 1-GPU profile scaled to the widest slab; "
                                  "slab fill time includes the wait for the left neighbour's first rows")
            if fill_max > 0 else None,
        }
        print(json.dumps(line), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


import json  # noqa: E402  (used by bench_main)
