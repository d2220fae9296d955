"""Chunk-sharded multi-GPU separation of one track (one process per GPU, RCCL over xGMI).

The reference has no distributed path (only a dead nn.DataParallel, inference.py:209-210).
Chunks of the chunker/OLA are independent given the mix, so:

* rank r takes the contiguous global chunk range [lo_r, hi_r) of the reference chunk plan -- the
  generic mode of inference_pytorch.py:85-163 (fades, border reflect pad) or the demucs mode of
  utils.py:371-445 (C = samplerate * segment, no fades / pad, ``counter += 1``) -- and runs
  gather -> forward -> windowed OLA into a LOCAL span buffer of result rows covering only the
  samples its chunks touch ([start(lo_r), end(hi_r - 1)) of the padded track);
* one ``gather`` of the fixed-size span buffers to rank 0 (RCCL, backend "nccl": point-to-point
  receives over rank 0's xGMI links) -- the only exchange; rank 0 sums the seams (C - step samples
  between neighbours) in rank order.  Only rank 0 assembles and finalises: the other ranks receive
  nothing (round 4 all-gathered every span to every rank, ~2.7 GB per rank for HTDemucs 30-min at
  world 8, thrown away by all but rank 0).  ``gather_to=None`` keeps the all-gather form for callers
  that want the stems on every rank;
* the counter is deterministic: rank 0 recomputes it for the whole plan with the same kernel and
  chunk order as the single-GPU path (``sesa_ola_accumulate_f32`` with no result rows), so it is
  bit-identical to it and is not exchanged; then ``result / counter`` is finalised.

The OWNED form (``demix_owned``, round 6; bench.py's multi-GPU line): no rank assembles the track.  Each rank
uploads only the mix samples its chunks read (``input_span``), sends the seam of its span buffer -- the C - step
samples its last chunks share with the next rank's first -- to that neighbour (``exchange_halos``: one RCCL
point-to-point message per neighbour pair, ~C x rows x 4 B), and finalises the output range its chunks start in
(``owned_ranges``), which it can copy to the host on its own PCIe link: the ranks' ranges tile the track.

Summation order at the seams differs from the reference's sequential chunk order only by the
grouping of fp32 additions (rank partial sums), ~1e-7 relative.
"""
import torch
import torch.distributed as dist

from .config import prefer_target_instrument
from .demix import chunk_plan, demucs_chunk_plan


def shard_ranges(n_chunks, world):
    per = -(-n_chunks // world)
    return [(min(r * per, n_chunks), min((r + 1) * per, n_chunks)) for r in range(world)]


def shard_plan(config, L, world, mode="generic"):
    """Host-side plan: flat chunk list [(start, seg, no_fade_in, no_fade_out)] (padded coordinates),
    per-rank chunk ranges and sample spans, chunk size C, padded length and border."""
    if mode == "demucs":
        C = int(config.training.samplerate * config.training.segment)
        flat = [(s, n, False, False) for s, n in demucs_chunk_plan(L, C, int(config.inference.num_overlap))]
        padded, border, L_pad = False, 0, L
    else:
        C = int(config.audio.chunk_size)
        padded, border, L_pad, batches, _ = chunk_plan(L, C, int(config.inference.num_overlap),
                                                       int(config.inference.batch_size))
        flat = [(s, n, ni_, no) for chunks, ni_, no in batches for (s, n) in chunks]
    ranges = shard_ranges(len(flat), world)
    spans = []
    for lo, hi in ranges:
        spans.append((0, 0) if lo >= hi else (flat[lo][0], max(s + n for s, n, _, _ in flat[lo:hi])))
    span_max = max(1, max(e - s for s, e in spans))
    return dict(mode=mode, chunk=C, padded=padded, border=border if padded else 0, L_pad=L_pad, flat=flat,
                ranges=ranges, spans=spans, span_max=span_max)


class _Windows:
    """The plan's windows on the device: generic mode -> the batch's faded window
    (inference_pytorch.py:151-155), demucs mode -> ones (utils.py:443-445)."""

    def __init__(self, plan, device):
        from .demix import _Windows as W
        self.ones = torch.ones(plan["chunk"], device=device, dtype=torch.float32) if plan["mode"] == "demucs" else None
        self.w = None if self.ones is not None else W(plan["chunk"], device)

    def pick(self, no_in, no_out):
        return self.ones if self.ones is not None else self.w.pick(no_in, no_out)


def _runs(group):
    """Consecutive runs of chunks sharing a window (== the reference's logical batches), in order."""
    j = 0
    while j < len(group):
        k = j
        while k < len(group) and group[k][2:] == group[j][2:]:
            k += 1
        yield j, k
        j = k


_SIDE_STREAMS = {}


def side_streams(device, n):
    """n side streams of `device`, created once per process and reused by every call: each stream keys
    its own model workspace (NativeModule.workspace), so fresh streams per call would grow that cache."""
    pool = _SIDE_STREAMS.setdefault(device.index, [])
    while len(pool) < n:
        pool.append(torch.cuda.Stream(device))
    return pool[:n]


def local_accumulate_device(config, model, mix_d, plan, rank, rows, exec_batch, streams=1):
    """gather -> forward -> OLA of this rank's chunks into a [rows, span_max] result buffer (HIP).

    ``streams`` > 1: consecutive forwards alternate between the current stream and side streams (each
    with its own input buffer and model workspace) so that one forward's memory-bound phases can overlap
    another's MFMA-bound ones; the OLA of every forward stays on the current stream, in chunk order,
    after an event on its forward's stream, so the result is bit-identical to streams = 1
    (tests/test_gpu_parity.py::test_side_streams_bit_identical).  (Rounds 4-5 refused streams > 1: the FFT
    kernels' SLP-packed complex arithmetic -- v_pk_*_f32 with a source op_sel -- computed wrong values while
    another stream's MFMA kernel shared their CUs; libsesa is now built without those instructions,
    tools/isa_guard.py)"""
    from . import ops
    C = plan["chunk"]
    n_ch = mix_d.shape[0]
    device = mix_d.device
    local = torch.zeros(rows, plan["span_max"], device=device, dtype=torch.float32)
    scratch = torch.zeros(plan["span_max"], device=device, dtype=torch.float32)   # counter: recomputed later
    lo, hi = plan["ranges"][rank]
    s0 = plan["spans"][rank][0]
    flat = plan["flat"]
    win = _Windows(plan, device)
    main = torch.cuda.current_stream(device)
    if not getattr(model, "multi_stream_ok", True):
        streams = 1            # (a model whose forwards are not bit-identical across streams)
    pool = [main] + side_streams(device, max(1, int(streams)) - 1)
    xbufs = [None] * len(pool)
    freed = [None] * len(pool)    # event on main after the OLA that consumed the stream's last forward
    for st in pool[1:]:
        st.wait_stream(main)      # the mix upload and buffer zeroing happen-before every side stream
    pos, gi = lo, 0
    while pos < hi:
        grp = flat[pos:min(hi, pos + exec_batch)]
        si = gi % len(pool)
        st = pool[si]
        if st is not main and freed[si] is not None:
            st.wait_event(freed[si])          # its input buffer / workspace are free again
        with torch.cuda.stream(st):
            if xbufs[si] is None or xbufs[si].shape[0] != len(grp):
                xbufs[si] = torch.empty(len(grp), n_ch, C, device=device, dtype=torch.float32)
            xbuf = xbufs[si]
            starts = [g[0] for g in grp]
            if plan["mode"] == "demucs":
                ops.chunk_gather_constant(mix_d, starts, C, out=xbuf)
            else:
                ops.chunk_gather(mix_d, plan["border"], starts, C, out=xbuf)
            y = model(xbuf).reshape(len(grp), rows, C)
        if st is not main:
            main.wait_stream(st)
            y.record_stream(main)
        for j, k in _runs(grp):
            ops.ola_accumulate(y[j:k], [g[0] - s0 for g in grp[j:k]], [g[1] for g in grp[j:k]],
                               win.pick(*grp[j][2:]), local, scratch)
        if st is not main:
            freed[si] = torch.cuda.Event()
            freed[si].record(main)
        pos += len(grp)
        gi += 1
    for st in pool[1:]:
        main.wait_stream(st)
    return local


def counter_device(plan, device):
    """The whole plan's counter (inference_pytorch.py:158 / utils.py:442,445), recomputed locally with
    the single-GPU kernel and chunk order: bit-identical on every rank, never exchanged."""
    from . import ops
    counter = torch.zeros(plan["L_pad"], device=device, dtype=torch.float32)
    win = _Windows(plan, device)
    flat = plan["flat"]
    for j, k in _runs(flat):
        ops.ola_counter(plan["chunk"], [g[0] for g in flat[j:k]], [g[1] for g in flat[j:k]],
                        win.pick(*flat[j][2:]), counter)
    return counter


def exchange_and_assemble(local, plan, rank, world, group=None, gather_to=0, simulate=False):
    """Gather the span buffers to rank ``gather_to`` (or all-gather them to every rank when it is None) and
    sum them into the full [rows, L_pad] result; ranks that receive nothing return None.  ``simulate``: a
    one-process rehearsal of rank ``rank``'s share of a ``world``-rank run (bench.py --rank-share): no
    collective, only this rank's span is assembled."""
    rows, span_max = local.shape
    local = local.contiguous()
    if world > 1 and not simulate:
        if gather_to is None:
            gathered = torch.empty(world * rows, span_max, device=local.device, dtype=local.dtype)
            dist.all_gather_into_tensor(gathered, local, group=group)
            gathered = list(gathered.view(world, rows, span_max))
        elif rank == gather_to:
            gathered = [torch.empty_like(local) for _ in range(world)]
            dist.gather(local, gathered, dst=gather_to if group is None else dist.get_global_rank(group, gather_to),
                        group=group)
        else:
            dist.gather(local, None, dst=gather_to if group is None else dist.get_global_rank(group, gather_to),
                        group=group)
            return None
    else:
        gathered = {rank: local} if simulate else [local]
    full = torch.zeros(rows, plan["L_pad"], device=local.device, dtype=local.dtype)
    for r, (s, e) in enumerate(plan["spans"]):
        if e > s and (not simulate or r == rank):
            full[:, s:e] += gathered[r][:, :e - s]
    return full


def owned_ranges(plan):
    """Padded-coordinate range [a_r, b_r) of the output each rank finalises in the owned form: consecutive non-empty
    ranks own from their first chunk's start to the next non-empty rank's (the first from 0, the last to L_pad);
    empty ranks own nothing.  None when some rank's span reaches past the next rank's owned range (a rank with fewer
    than overlap - 1 chunks): then only the gather form assembles the seams."""
    ne = [r for r, (lo, hi) in enumerate(plan["ranges"]) if hi > lo]
    own = [(0, 0)] * len(plan["ranges"])
    for i, r in enumerate(ne):
        a = 0 if i == 0 else plan["spans"][r][0]
        b = plan["L_pad"] if i + 1 == len(ne) else plan["spans"][ne[i + 1]][0]
        own[r] = (a, b)
    for i in range(len(ne) - 1):
        if plan["spans"][ne[i]][1] > own[ne[i + 1]][1]:
            return None
    return own


def input_span(plan, rank, L):
    """Unpadded sample range [lo, hi) of the mix rank ``rank``'s chunks read (the reflect border of the track's ends
    included): the part of a host-resident track that rank has to upload.  (0, 0) for an empty rank."""
    lo_c, hi_c = plan["ranges"][rank]
    if lo_c >= hi_c:
        return 0, 0
    s, e = plan["spans"][rank]
    b = plan["border"]
    lo = max(0, s - b - 1)
    hi = L if e - b > L else e - b + 1
    if s - b < 0:       # reflect pad of the track's start reads samples 1 .. b
        hi = max(hi, min(L, b + 1))
    if e - b > L:       # ... and of its end L - 2 .. L - 1 - b
        lo = min(lo, max(0, L - b - 2))
    return lo, min(hi, L)


def exchange_halos(local, plan, rank, group=None):
    """Owned form's only exchange: every non-empty rank sends the tail of its span buffer that overlaps the next
    non-empty rank's span (C - step samples, the seam) to that rank, which adds it in -- RCCL point-to-point
    (gloo on CPU), one message per neighbour pair."""
    ne = [r for r, (lo, hi) in enumerate(plan["ranges"]) if hi > lo]
    if rank not in ne:
        return local
    i = ne.index(rank)
    ops_ = []
    recv = None
    if i + 1 < len(ne):
        nx = ne[i + 1]
        s, e = plan["spans"][rank]
        t0 = plan["spans"][nx][0] - s
        if e - s > t0:
            tail = local[:, t0:e - s].contiguous()
            ops_.append(dist.P2POp(dist.isend, tail, nx if group is None else dist.get_global_rank(group, nx), group))
    if i > 0:
        pv = ne[i - 1]
        n = plan["spans"][pv][1] - plan["spans"][rank][0]
        if n > 0:
            recv = torch.empty(local.shape[0], n, device=local.device, dtype=local.dtype)
            ops_.append(dist.P2POp(dist.irecv, recv, pv if group is None else dist.get_global_rank(group, pv), group))
    for w in (dist.batch_isend_irecv(ops_) if ops_ else []):
        w.wait()
    if recv is not None:
        local[:, :recv.shape[1]] += recv
    return local


def demix_owned(config, model, mix_d, device=None, rank=None, world=None, exec_batch=8, group=None, local_fn=None,
                finalize_fn=None, counter_fn=None, mode="generic", streams=1, simulate=False):
    """The owned form of the chunk shard: each rank finalises only the part of the output its chunks start in
    (``owned_ranges``) after one halo exchange with its neighbours, so no rank gathers the track: returns
    (est [n_instr, 2, hi - lo], lo, hi) -- the unpadded sample range [lo, hi) of the stems this rank holds; the
    ranks' ranges tile [0, L).  The mix need only be resident over ``input_span`` (the rest of ``mix_d`` is not
    read).  Falls back to None when the plan has a rank too short for a single seam (``owned_ranges``); callers
    then use ``demix_sharded``."""
    rank = dist.get_rank(group) if rank is None else rank
    world = dist.get_world_size(group) if world is None else world
    instruments = list(config.training.instruments) if mode == "demucs" else prefer_target_instrument(config)
    ni = len(instruments)
    n_ch, L = mix_d.shape
    rows = ni * n_ch
    if L == 0:
        return torch.zeros(ni, n_ch, 0, device=mix_d.device, dtype=torch.float32), 0, 0
    plan = shard_plan(config, L, world, mode)
    own = owned_ranges(plan)
    if own is None:
        return None
    if local_fn is None:
        local = local_accumulate_device(config, model, mix_d, plan, rank, rows, exec_batch, streams)
    else:
        local = local_fn(config, model, mix_d, plan, rank, rows)
    if world > 1 and not simulate:
        local = exchange_halos(local, plan, rank, group)
    a, b = own[rank]
    bd = plan["border"]
    lo, hi = max(a, bd), min(b, plan["L_pad"] - bd)        # padded range that survives the border crop
    if hi <= lo:
        return torch.zeros(ni, n_ch, 0, device=mix_d.device, dtype=torch.float32), 0, 0
    s0 = plan["spans"][rank][0]
    counter = counter_device(plan, mix_d.device) if counter_fn is None else counter_fn(plan)
    seg = local[:, lo - s0:hi - s0].contiguous()
    if finalize_fn is None:
        from . import ops
        est = ops.ola_finalize(seg, counter[lo:hi].contiguous(), 0)
    else:
        est = finalize_fn(seg, counter[lo:hi].contiguous(), 0)
    return est.reshape(ni, n_ch, hi - lo), lo - bd, hi - bd


def demix_sharded(config, model, mix_d, device=None, rank=None, world=None, exec_batch=8, group=None,
                  local_fn=None, finalize_fn=None, counter_fn=None, mode="generic", streams=1, gather_to=0,
                  simulate=False):
    """Separate the device-resident mix [2, L] with chunks sharded across the process group.
    ``mode``: "generic" (inference_pytorch.demix_pytorch_optimized / utils.demix generic) or
    "demucs" (utils.demix for model_type 'htdemucs').  Returns est [n_instr, 2, L] on rank ``gather_to``
    (every rank when ``gather_to`` is None) and None on the others.  ``simulate``: run only rank ``rank``'s
    share of a ``world``-rank plan in this one process, no collective (the per-rank compute ceiling of a
    multi-GPU run, measured on one GPU; its output is that share's samples only).
    ``local_fn`` / ``counter_fn`` / ``finalize_fn`` exist so the CPU test-suite can drive the
    sharding + collective + assembly with the oracle's OLA (gloo); the product path uses the HIP ops."""
    rank = dist.get_rank(group) if rank is None else rank
    world = dist.get_world_size(group) if world is None else world
    instruments = list(config.training.instruments) if mode == "demucs" else prefer_target_instrument(config)
    ni = len(instruments)
    n_ch, L = mix_d.shape
    rows = ni * n_ch
    if L == 0:
        if world > 1 and not simulate and gather_to is not None and rank != gather_to:
            return None   # (the gather contract: only rank gather_to holds the result)
        return torch.zeros(ni, n_ch, 0, device=mix_d.device, dtype=torch.float32)
    plan = shard_plan(config, L, world, mode)
    if local_fn is None:
        local = local_accumulate_device(config, model, mix_d, plan, rank, rows, exec_batch, streams)
    else:
        local = local_fn(config, model, mix_d, plan, rank, rows)
    full = exchange_and_assemble(local, plan, rank, world, group, gather_to, simulate)
    if full is None:
        return None
    counter = counter_device(plan, mix_d.device) if counter_fn is None else counter_fn(plan)
    if finalize_fn is None:
        from . import ops
        est = ops.ola_finalize(full.contiguous(), counter, plan["border"])
    else:
        est = finalize_fn(full, counter, plan["border"])
    return est.reshape(ni, n_ch, L)
