"""World-size-2 (and 3) gloo test of the chunk-shard path (sesa/parallel.py) on CPU: shard plan,
span all_gather and seam assembly, with the oracle's chunker/OLA standing in for the HIP ops
(the product path itself refuses CPU tensors).  Compared with the single-process oracle demix."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import CONFIGS

L_TRACK = 300000


class StandIn:
    def __call__(self, x):
        return torch.stack([x, -0.5 * x + 0.01 * torch.roll(x, 7, -1)], 1)


def _cfg(bs):
    from sesa.config import load_config
    c = load_config("mdx23c", os.path.join(CONFIGS, "config_mdx23c_small.yaml"))
    c.inference.batch_size = bs
    return c


def _mix():
    rng = np.random.default_rng(3)
    return (0.1 * rng.standard_normal((2, L_TRACK))).astype(np.float32)


def _plan_windows(config, plan):
    from oracle.demix import windowing_array
    C = plan["chunk"]
    fade = C // 10
    base = windowing_array(C, fade)

    def win(no_in, no_out):
        if plan["mode"] == "demucs":
            return np.ones(C, np.float32)
        w = base.copy()
        if no_in:
            w[:fade] = 1
        elif no_out:
            w[-fade:] = 1
        return w
    return win


def cpu_local(config, model, mix, plan, rank, rows):
    from oracle.demix import extract_chunk
    C = plan["chunk"]
    mixn = mix.numpy()
    b = plan["border"]
    mix_pad = np.pad(mixn, ((0, 0), (b, b)), mode="reflect") if b else mixn
    local = np.zeros((rows, plan["span_max"]), np.float32)
    lo, hi = plan["ranges"][rank]
    s0 = plan["spans"][rank][0]
    win = _plan_windows(config, plan)
    for (s, n, no_in, no_out) in plan["flat"][lo:hi]:
        if plan["mode"] == "demucs":
            part = mixn[:, s:s + C]
            x = np.pad(part, ((0, 0), (0, C - part.shape[1])))
        else:
            x = extract_chunk(mix_pad, s, C)
        y = model(torch.from_numpy(x)[None]).numpy().reshape(rows, C)
        local[:, s - s0:s - s0 + n] += y[:, :n] * win(no_in, no_out)[:n]
    return torch.from_numpy(local)


def make_cpu_counter(config):
    def counter_fn(plan):
        win = _plan_windows(config, plan)
        c = np.zeros(plan["L_pad"], np.float32)
        for (s, n, no_in, no_out) in plan["flat"]:
            c[s:s + n] += win(no_in, no_out)[:n]
        return torch.from_numpy(c)
    return counter_fn


def cpu_finalize(result, counter, border):
    with np.errstate(divide="ignore", invalid="ignore"):
        est = (result / counter).numpy()
    np.nan_to_num(est, copy=False, nan=0.0)
    if border:
        est = est[:, border:-border]
    return torch.from_numpy(np.ascontiguousarray(est))


def _demucs_cfg():
    from sesa.config import wrap
    return wrap({"training": {"samplerate": 1000, "segment": 40, "instruments": ["vocals", "other"]},
                 "inference": {"num_overlap": 4, "batch_size": 2}})


class StandIn2:
    """A second, different stand-in member (ensemble tests)."""

    def __call__(self, x):
        return torch.stack([0.7 * x + 0.02 * torch.roll(x, -3, -1), 0.3 * x], 1)


def _worker(rank, world, port, bs, q, mode="generic", L=L_TRACK):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sesa.parallel import demix_sharded
        cfg = _demucs_cfg() if mode == "demucs" else _cfg(bs)
        mix = torch.from_numpy(_mix()[:, :L])
        if mode == "ensemble":
            from oracle.ensemble import blend
            from sesa.ensemble import ensemble_separate
            hooks = dict(local_fn=cpu_local, finalize_fn=cpu_finalize, counter_fn=make_cpu_counter(cfg))
            out, stems = ensemble_separate([(cfg, StandIn()), (cfg, StandIn2())], mix, "vocals", "avg_wave",
                                           weights=[0.6, 0.4], rank=rank, world=world, demix_hooks=hooks,
                                           blend_fn=lambda x, m, w, b: torch.from_numpy(blend(x.numpy(), m, w, b)))
            est = out
        else:
            est = demix_sharded(cfg, StandIn(), mix, rank=rank, world=world,
                                local_fn=cpu_local, finalize_fn=cpu_finalize, counter_fn=make_cpu_counter(cfg),
                                mode="generic" if mode == "allgather" else mode,
                                gather_to=None if mode == "allgather" else 0)
            if mode == "allgather":           # every rank holds the stems; they must agree with rank 0's
                ref0 = est.clone()
                dist.broadcast(ref0, 0)
                assert torch.equal(est, ref0)
        if rank == 0:
            q.put(est.numpy())
        elif mode != "allgather":
            assert est is None                # gather to rank 0: the other ranks receive nothing
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,bs", [(2, 1), (3, 2)])
def test_chunk_shard_matches_single_process(world, bs):
    from oracle.demix import demix as odemix
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    pc = mp.start_processes(_worker, args=(world, port, bs, q), nprocs=world, join=False, start_method="spawn")
    est = q.get()  # read before joining: the 4.8 MB result would otherwise block the pipe
    while not pc.join(timeout=120):
        pass
    ref = odemix(_cfg(bs), StandIn(), _mix(), batch_size=bs)
    ref = np.stack([ref["vocals"], ref["other"]])
    assert est.shape == ref.shape
    # seams are summed per rank (fp32 regrouping only): ~1e-7 relative
    assert np.abs(est - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("world", [2, 3])
def test_demucs_mode_shard_matches_single_process(world):
    """utils.demix demucs mode (model_type 'htdemucs', utils.py:371-445) sharded over gloo ranks vs the
    single-process oracle restatement (pinned to the reference by tests/test_demucs_mode.py)."""
    from oracle.demix import demix_demucs_mode
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    pc = mp.start_processes(_worker, args=(world, port, 1, q, "demucs"), nprocs=world, join=False,
                            start_method="spawn")
    est = q.get()
    while not pc.join(timeout=120):
        pass
    cfg = _demucs_cfg()
    ref = demix_demucs_mode(cfg, StandIn(), _mix())
    ref = np.stack([ref["vocals"], ref["other"]])
    assert est.shape == ref.shape
    assert np.abs(est - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max())


def test_shard_plan_covers_every_chunk_once():
    from sesa.parallel import shard_plan
    c = _cfg(1)
    for world in (1, 2, 3, 8):
        p = shard_plan(c, L_TRACK, world) if world % 2 else shard_plan(_demucs_cfg(), L_TRACK, world, "demucs")
        covered = [i for lo, hi in p["ranges"] for i in range(lo, hi)]
        assert covered == list(range(len(p["flat"])))
        for (lo, hi), (s, e) in zip(p["ranges"], p["spans"]):
            for (st, n, _, _) in p["flat"][lo:hi]:
                assert s <= st and st + n <= e


def _run_world(world, mode, bs=1, L=L_TRACK):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    pc = mp.start_processes(_worker, args=(world, port, bs, q, mode, L), nprocs=world, join=False,
                            start_method="spawn")
    est = q.get()
    while not pc.join(timeout=180):
        pass
    return est


# World 8 (the driver's scaling node): a 13-chunk track (97 000 samples of the reduced config, chunk 64 512 at
# overlap 4) gives ranges of 2 chunks and an EMPTY rank 7 (sesa/parallel.py shard_ranges); the demucs-mode
# plan and the ensemble member loop (one all_gather per member, then the blend) at the same world size.
L13 = 97000


def test_world8_generic_with_empty_rank():
    from oracle.demix import demix as odemix
    from sesa.parallel import shard_plan
    p = shard_plan(_cfg(1), L13, 8)
    assert len(p["flat"]) == 13 and p["ranges"][7][0] == p["ranges"][7][1]
    est = _run_world(8, "generic", L=L13)
    ref = odemix(_cfg(1), StandIn(), _mix()[:, :L13], batch_size=1)
    ref = np.stack([ref["vocals"], ref["other"]])
    assert est.shape == ref.shape
    assert np.abs(est - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max())


def test_world8_demucs_mode():
    from oracle.demix import demix_demucs_mode
    est = _run_world(8, "demucs")
    ref = demix_demucs_mode(_demucs_cfg(), StandIn(), _mix())
    ref = np.stack([ref["vocals"], ref["other"]])
    assert est.shape == ref.shape
    assert np.abs(est - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max())


def test_world8_ensemble_two_members():
    """ensemble_separate over 8 gloo ranks (each member chunk-sharded, its own all_gather) + avg_wave blend
    with weights, against the single-process oracle demix of each member and the oracle blend."""
    from oracle.demix import demix as odemix
    from oracle.ensemble import blend
    est = _run_world(8, "ensemble", L=L13)
    mix = _mix()[:, :L13]
    v1 = odemix(_cfg(1), StandIn(), mix, batch_size=1)["vocals"]
    v2 = odemix(_cfg(1), StandIn2(), mix, batch_size=1)["vocals"]
    ref = blend(np.stack([v1, v2]), "avg_wave", [0.6, 0.4], 32768)
    assert est.shape == ref.shape
    assert np.abs(est - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max())


def test_allgather_form_matches_single_process():
    """gather_to=None: the all-gather form (stems on every rank), world 3."""
    from oracle.demix import demix as odemix
    est = _run_world(3, "allgather")
    ref = odemix(_cfg(1), StandIn(), _mix(), batch_size=1)
    ref = np.stack([ref["vocals"], ref["other"]])
    assert np.abs(est - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("world", [3, 8])
def test_rank_share_rehearsal_sums_to_whole(world):
    """simulate=True (bench.py --rank-share): each rank's share run alone in one process, no collective.
    The shares' finalised outputs sum to the whole track's (finalisation is a division by the shared
    counter), so the per-rank rehearsal does exactly its share of the work."""
    from oracle.demix import demix as odemix
    from sesa.parallel import demix_sharded, shard_plan
    cfg = _cfg(1)
    mix = torch.from_numpy(_mix())
    total = None
    for r in range(world):
        est = demix_sharded(cfg, StandIn(), mix, rank=r, world=world, local_fn=cpu_local, finalize_fn=cpu_finalize,
                            counter_fn=make_cpu_counter(cfg), simulate=True)
        total = est.numpy().astype(np.float64) if total is None else total + est.numpy()
    ref = odemix(cfg, StandIn(), _mix(), batch_size=1)
    ref = np.stack([ref["vocals"], ref["other"]])
    assert np.abs(total - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max())
    plan = shard_plan(cfg, L_TRACK, world)
    assert sum(hi - lo for lo, hi in plan["ranges"]) == len(plan["flat"])


# ---- owned form (round 6): halo exchange between neighbours, each rank finalises its own range ----------------
def _owned_worker(rank, world, port, q, mode, L):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sesa.parallel import demix_owned, input_span, shard_plan
        cfg = _demucs_cfg() if mode == "demucs" else _cfg(1)
        full = torch.from_numpy(_mix()[:, :L])
        # only this rank's input span is present: everything else is NaN, so a read outside it would show
        plan = shard_plan(cfg, L, world, mode)
        lo, hi = input_span(plan, rank, L)
        mix = torch.full_like(full, float("nan"))
        mix[:, lo:hi] = full[:, lo:hi]
        res = demix_owned(cfg, StandIn(), mix, rank=rank, world=world, local_fn=cpu_local, finalize_fn=cpu_finalize,
                          counter_fn=make_cpu_counter(cfg), mode=mode)
        est, a, b = res
        q.put((rank, a, b, est.numpy()))
    finally:
        dist.destroy_process_group()


def _run_owned(world, mode, L):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    pc = mp.start_processes(_owned_worker, args=(world, port, q, mode, L), nprocs=world, join=False,
                            start_method="spawn")
    parts = sorted(q.get() for _ in range(world))
    while not pc.join(timeout=180):
        pass
    return parts


@pytest.mark.parametrize("world,mode,L", [(2, "generic", L_TRACK), (3, "generic", L_TRACK), (3, "demucs", L_TRACK),
                                          (8, "demucs", L_TRACK)])
def test_owned_form_tiles_and_matches_single_process(world, mode, L):
    """demix_owned over gloo ranks: every rank uploads only its input_span (NaN elsewhere), exchanges one seam
    with each neighbour and finalises its owned range; the ranges tile [0, L) and the stitched stems equal the
    single-process oracle demix (fp32 seam regrouping only)."""
    from oracle.demix import demix as odemix, demix_demucs_mode
    parts = _run_owned(world, mode, L)
    assert parts[0][1] == 0 and parts[-1][2] == L
    for (_, a, b, _), (_, a2, _, _) in zip(parts, parts[1:]):
        assert b == a2 or (a == b)
    est = np.concatenate([p[3] for p in parts if p[2] > p[1]], axis=-1)
    if mode == "demucs":
        ref = demix_demucs_mode(_demucs_cfg(), StandIn(), _mix()[:, :L])
    else:
        ref = odemix(_cfg(1), StandIn(), _mix()[:, :L], batch_size=1)
    ref = np.stack([ref["vocals"], ref["other"]])
    assert est.shape == ref.shape and np.isfinite(est).all()
    assert np.abs(est - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max())


def test_owned_ranges_refuse_short_ranks():
    """A rank with fewer chunks than one seam spans (13 chunks over 8 ranks: 2 per rank at overlap 4) makes the
    owned form unavailable (None) -- callers then gather."""
    from sesa.parallel import owned_ranges, shard_plan
    assert owned_ranges(shard_plan(_cfg(1), L13, 8)) is None
    assert owned_ranges(shard_plan(_cfg(1), L_TRACK, 2)) is not None
