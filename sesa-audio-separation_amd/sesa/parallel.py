"""Chunk-sharded multi-GPU separation of one track (one process per GPU, RCCL over xGMI).

The reference has no distributed path (only a dead nn.DataParallel, inference.py:209-210).
Chunks of the chunker/OLA (inference_pytorch.py:123-159) are independent given the mix, so:

* rank r takes the contiguous global chunk range [lo_r, hi_r) of the reference chunk plan and
  runs gather -> forward -> windowed OLA into a LOCAL span buffer covering only the samples its
  chunks touch ([start(lo_r), end(hi_r - 1)) of the padded track): result rows + a counter row;
* one ``all_gather_into_tensor`` of the fixed-size span buffers (RCCL, backend "nccl") -- the only
  exchange; the seams (C - step samples between neighbours) are summed in rank order and
  ``result / counter`` is finalised.

Summation order at the seams differs from the reference's sequential chunk order only by the
grouping of fp32 additions (rank partial sums), ~1e-7 relative.
"""
import torch
import torch.distributed as dist

from .config import prefer_target_instrument
from .demix import chunk_plan


def shard_ranges(n_chunks, world):
    per = -(-n_chunks // world)
    return [(min(r * per, n_chunks), min((r + 1) * per, n_chunks)) for r in range(world)]


def shard_plan(config, L, world):
    """Host-side plan: flat chunk list [(start, seg, no_fade_in, no_fade_out)], per-rank chunk ranges
    and sample spans (padded coordinates)."""
    C = int(config.audio.chunk_size)
    padded, border, L_pad, batches, _ = chunk_plan(L, C, int(config.inference.num_overlap),
                                                   int(config.inference.batch_size))
    flat = [(s, n, ni_, no) for chunks, ni_, no in batches for (s, n) in chunks]
    ranges = shard_ranges(len(flat), world)
    spans = []
    for lo, hi in ranges:
        spans.append((0, 0) if lo >= hi else (flat[lo][0], max(s + n for s, n, _, _ in flat[lo:hi])))
    span_max = max(1, max(e - s for s, e in spans))
    return dict(padded=padded, border=border if padded else 0, L_pad=L_pad, flat=flat, ranges=ranges,
                spans=spans, span_max=span_max)


def local_accumulate_device(config, model, mix_d, plan, rank, rows, exec_batch):
    """gather -> forward -> OLA of this rank's chunks into a [rows + 1, span_max] buffer (HIP)."""
    from . import ops
    from .demix import _Windows
    C = int(config.audio.chunk_size)
    n_ch = mix_d.shape[0]
    device = mix_d.device
    local = torch.zeros(rows + 1, plan["span_max"], device=device, dtype=torch.float32)
    lo, hi = plan["ranges"][rank]
    s0 = plan["spans"][rank][0]
    flat = plan["flat"]
    win = _Windows(C, device)
    xbuf = None
    pos = lo
    while pos < hi:
        grp = flat[pos:min(hi, pos + exec_batch)]
        if xbuf is None or xbuf.shape[0] != len(grp):
            xbuf = torch.empty(len(grp), n_ch, C, device=device, dtype=torch.float32)
        ops.chunk_gather(mix_d, plan["border"], [g[0] for g in grp], C, out=xbuf)
        y = model(xbuf).reshape(len(grp), rows, C)
        j = 0
        while j < len(grp):
            k = j
            while k < len(grp) and grp[k][2:] == grp[j][2:]:
                k += 1
            ops.ola_accumulate(y[j:k], [g[0] - s0 for g in grp[j:k]], [g[1] for g in grp[j:k]],
                               win.pick(*grp[j][2:]), local[:rows], local[rows])
            j = k
        pos += len(grp)
    return local


def exchange_and_assemble(local, plan, rank, world, group=None):
    """All-gather the span buffers and sum them into the full [rows + 1, L_pad] (result, counter)."""
    rows1, span_max = local.shape
    if world > 1:
        gathered = torch.empty(world * rows1, span_max, device=local.device, dtype=local.dtype)
        dist.all_gather_into_tensor(gathered, local.contiguous(), group=group)
        gathered = gathered.view(world, rows1, span_max)
    else:
        gathered = local[None]
    full = torch.zeros(rows1, plan["L_pad"], device=local.device, dtype=local.dtype)
    for r, (s, e) in enumerate(plan["spans"]):
        if e > s:
            full[:, s:e] += gathered[r, :, :e - s]
    return full


def demix_sharded(config, model, mix_d, device=None, rank=None, world=None, exec_batch=8, group=None,
                  local_fn=None, finalize_fn=None):
    """Separate the device-resident mix [2, L] with chunks sharded across the process group.
    Returns est [n_instr, 2, L] on every rank.  ``local_fn`` / ``finalize_fn`` exist so the CPU
    test-suite can drive the sharding + collective + assembly with the oracle's OLA (gloo);
    the product path uses the HIP ops."""
    rank = dist.get_rank(group) if rank is None else rank
    world = dist.get_world_size(group) if world is None else world
    ni = len(prefer_target_instrument(config))
    n_ch, L = mix_d.shape
    rows = ni * n_ch
    if L == 0:
        return torch.zeros(ni, n_ch, 0, device=mix_d.device, dtype=torch.float32)
    plan = shard_plan(config, L, world)
    if local_fn is None:
        local = local_accumulate_device(config, model, mix_d, plan, rank, rows, exec_batch)
    else:
        local = local_fn(config, model, mix_d, plan, rank, rows)
    full = exchange_and_assemble(local, plan, rank, world, group)
    if finalize_fn is None:
        from . import ops
        est = ops.ola_finalize(full[:rows].contiguous(), full[rows].contiguous(), plan["border"])
    else:
        est = finalize_fn(full[:rows], full[rows], plan["border"])
    return est.reshape(ni, n_ch, L)
