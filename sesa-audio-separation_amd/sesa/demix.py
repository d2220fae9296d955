"""Device-resident chunker + windowed overlap-add.

Drop-in for ``inference_pytorch.demix_pytorch_optimized`` (/root/reference/inference_pytorch.py:55-186)
and the generic mode of ``utils.demix`` (utils.py:330-477).  Same parameters, same return value
(``{instrument: np.ndarray[2, L] f32}``), same ``[SESA_PROGRESS]N`` stdout lines, same window and
counter quirks -- but the mix is uploaded once, chunks are gathered on the device, the model runs
``exec_batch`` chunks per launch, and result/counter accumulate in HBM; the only D2H copy is the
final stems.

The *logical* batch (``config.inference.batch_size``) still decides the window fix-ups exactly as
in the reference (:145-155); the *execution* batch is independent of it (InstanceNorm is
per-instance, so grouping chunks differently does not change any chunk's output).
"""
import contextlib
import math

import numpy as np
import torch

from . import ops
from .config import prefer_target_instrument


def windowing_array(chunk_size, fade_size):
    """utils._getWindowingArray (utils.py:295-327): torch.linspace fades, float32."""
    w = torch.ones(chunk_size)
    w[-fade_size:] = torch.linspace(1, 0, fade_size)
    w[:fade_size] = torch.linspace(0, 1, fade_size)
    return w


def flat_plan(batches):
    return [c for chunks, _, _ in batches for c in chunks]


def chunk_plan(L, chunk_size, num_overlap, batch_size):
    """Loop control of inference_pytorch.py:115-163.  Returns (padded, border, L_pad, batches,
    progress) with batches = [(chunks[(start, seg_len)], no_fade_in, no_fade_out)] and progress =
    the list of (chunk_index_after_which_printed, percent) lines the reference prints."""
    step = chunk_size // num_overlap
    border = chunk_size - step
    padded = L > 2 * border and border > 0
    L_pad = L + 2 * border if padded else L
    batches, cur, progress = [], [], []
    i, last, idx = 0, -1, 0
    while i < L_pad:
        seg = min(chunk_size, L_pad - i)
        cur.append((i, seg))
        i += step
        if len(cur) >= batch_size or i >= L_pad:
            no_in = i - step == 0
            batches.append((list(cur), no_in, (not no_in) and i >= L_pad))
            cur = []
        pct = int((i / L_pad) * 100)
        if pct > last:
            last = pct
            progress.append((idx, pct))
        idx += 1
    return padded, border, L_pad, batches, progress


# Chunks per native forward, per model class (measured on MI355X, profiles/r01_bench_*): larger
# batches amortise per-launch tails until the workspace or the gain runs out.
# chunks per forward at most (288 GB of HBM: the workspace check in plan_exec_batch still halves these where memory is
# short).  Round 5 same-box sweep (profiles/r05_n_bench_*.json): BS-Roformer 4 -> 16 +1.9 %, SCNet 48 -> 96 +3.9 %,
# HTDemucs 32 -> 48 +1.7 % (64: the same); MDX23C 57 -> 85 per forward +0.75 % (noise level; an explicit cap of 96
# would trip the half-free-HBM check at the vocals config's 1.7 GB per chunk), so it stays 64.
# (round 5, same-box A/B on the final kernels: HTDemucs 14 x 48 -> 11 x 61 chunks per forward +1.8 %,
# profiles/r05_ad_*.  MDX23C stays at 64: 2 x 85 measured +0.8 % over 3 x 57 with an explicit batch, but its workspace
# is over the half-free-HBM guard below, which halves cap 96 to 4 x 43 -- 0.6 % slower than 3 x 57, profiles/r05_ae_*)
EXEC_CAP = {"TFC_TDF_net": 64, "BSRoformer": 16, "MelBandRoformer": 16, "SCNet": 96, "HTDemucs": 64}


def unwrap_model(model):
    """The network behind a backend (HipBackend.compiled_model / .model), else ``model`` itself."""
    for attr in ("compiled_model", "model"):
        inner = getattr(model, attr, None)
        if inner is not None and not isinstance(inner, (str, bytes)) and callable(inner):
            return inner
    return model


def plan_exec_batch(model, n_chunks, chunk, device=None, world=1, cap=None, streams=1):
    """Execution batch for ``n_chunks`` chunks of length ``chunk`` spread over ``world`` ranks: the
    model's cap (EXEC_CAP), halved while its workspace would exceed half the free HBM, then balanced
    so a rank's last forward is not a small remainder (169 chunks at cap 64 -> 3 forwards of 57).
    ``model`` may be the network or a backend wrapping it (HipBackend: the CLI and utils.demix pass
    the backend), so the CLI plans the same batch as bench.py."""
    model = unwrap_model(model)
    cap = int(cap or EXEC_CAP.get(type(model).__name__, 8))
    if hasattr(model, "workspace_bytes") and torch.cuda.is_available():
        try:
            free, _ = torch.cuda.mem_get_info(device)
            while cap > 1 and model.workspace_bytes(cap, chunk) * max(1, streams) > 0.5 * free:
                cap //= 2
        except Exception:  # noqa: BLE001 -- planning only; the forward itself reports real errors
            pass
    local = -(-max(1, n_chunks) // max(1, world))
    return max(1, -(-local // max(1, -(-local // cap))))


class _Windows:
    def __init__(self, chunk_size, device):
        fade = chunk_size // 10
        base = windowing_array(chunk_size, fade)
        w_in = base.clone()
        w_in[:fade] = 1
        w_out = base.clone()
        w_out[-fade:] = 1
        self.normal = base.to(device)
        self.no_in = w_in.to(device)
        self.no_out = w_out.to(device)

    def pick(self, no_in, no_out):
        return self.no_in if no_in else (self.no_out if no_out else self.normal)


# forwards in flight in demix_device (consecutive execution batches alternate between the current stream and side
# streams; the OLA stays on the current stream in chunk order, so the stems are bit-identical to one stream for the
# models whose forwards are -- NativeModule.multi_stream_ok).  Same box, bench.py --streams 1 vs 2: HTDemucs +4.6 %,
# MDX23C +1.4 % (profiles/r06_streams_ab.txt)
DEMIX_STREAMS = 2


def demix_device(config, model, mix, device, exec_batch=None, progress=True, chunk_range=None,
                 instruments=None, streams=None):
    """Core device loop.  ``mix`` is a host array [2, L] or a device tensor.  Returns the
    device tensor est [n_instr, 2, L] (after nan_to_num and border crop).

    ``streams`` (default DEMIX_STREAMS): execution batches in flight on separate HIP streams; the native forwards
    are re-entrant per stream (include/sesa.h) and the OLA runs on the current stream in chunk order, so the result
    does not depend on it.

    ``chunk_range`` = (first, last) restricts the work to a contiguous range of global chunk
    indices (multi-GPU chunk sharding, sesa/parallel.py); the caller then receives the raw
    (result, counter, plan) partial sums instead of the finalized estimate.
    """
    C = int(config.audio.chunk_size)
    ov = int(config.inference.num_overlap)
    bs = int(config.inference.batch_size)
    if instruments is None:
        instruments = prefer_target_instrument(config)
    ni = len(instruments)
    if isinstance(mix, torch.Tensor):
        mix_d = mix.to(device=device, dtype=torch.float32).contiguous()
    else:
        mix_d = torch.from_numpy(np.ascontiguousarray(mix, dtype=np.float32)).to(device, non_blocking=False)
    n_ch, L = mix_d.shape
    if L == 0:  # the reference loop never runs and returns empty stems (result/counter of length 0)
        if chunk_range is not None:
            return (torch.zeros(ni * n_ch, 0, device=device), torch.zeros(0, device=device), (False, 0, 0))
        return torch.zeros(ni, n_ch, 0, device=device, dtype=torch.float32)
    padded, border, L_pad, batches, prog = chunk_plan(L, C, ov, bs)
    streams = max(1, int(DEMIX_STREAMS if streams is None else streams)) if torch.device(device).type == "cuda" else 1
    if not getattr(model, "multi_stream_ok", True):
        streams = 1            # (a model whose forwards are not bit-identical across streams)
    E = exec_batch or getattr(model, "exec_batch", None) or plan_exec_batch(model, len(flat_plan(batches)), C,
                                                                            device, streams=streams)
    win = _Windows(C, device)
    result = torch.zeros(ni * n_ch, L_pad, device=device, dtype=torch.float32)
    counter = torch.zeros(L_pad, device=device, dtype=torch.float32)
    # flatten chunks with their logical-batch window
    flat = []
    for chunks, no_in, no_out in batches:
        for (s, n) in chunks:
            flat.append((s, n, no_in, no_out))
    lo, hi = (0, len(flat)) if chunk_range is None else chunk_range
    prog_at = dict(prog)
    pool, xbufs, freed = [None], [None], [None]
    if streams > 1:
        from .parallel import side_streams
        main = torch.cuda.current_stream(device)
        pool = [main] + side_streams(device, streams - 1)
        xbufs, freed = [None] * len(pool), [None] * len(pool)
        for st in pool[1:]:
            st.wait_stream(main)      # the mix upload and the zeroed buffers happen-before every side stream
    pos, gi = lo, 0
    while pos < hi:
        group = flat[pos:min(hi, pos + E)]
        starts = [g[0] for g in group]
        si = gi % len(pool)
        st = pool[si]
        side = st is not None and st is not pool[0]
        if side and freed[si] is not None:
            st.wait_event(freed[si])  # its input buffer / workspace are free again
        with torch.cuda.stream(st) if side else contextlib.nullcontext():
            if xbufs[si] is None or xbufs[si].shape[0] != len(group):
                xbufs[si] = torch.empty(len(group), n_ch, C, device=device, dtype=torch.float32)
            xbuf = xbufs[si]
            ops.chunk_gather(mix_d, border if padded else 0, starts, C, out=xbuf)
            y = model(xbuf)
            y = y.reshape(len(group), ni * n_ch, C)
        if side:
            pool[0].wait_stream(st)
            y.record_stream(pool[0])
        # OLA per run of equal windows (== per logical batch), in chunk order
        j = 0
        while j < len(group):
            k = j
            while k < len(group) and group[k][2:] == group[j][2:]:
                k += 1
            w = win.pick(*group[j][2:])
            ops.ola_accumulate(y[j:k], [g[0] for g in group[j:k]], [g[1] for g in group[j:k]], w, result, counter)
            j = k
        if side:
            freed[si] = torch.cuda.Event()
            freed[si].record(pool[0])
        if progress:
            for ci in range(pos, pos + len(group)):
                if ci in prog_at:
                    print(f"[SESA_PROGRESS]{prog_at[ci]}", flush=True)
        pos += len(group)
        gi += 1
    for st in pool[1:]:
        pool[0].wait_stream(st)
    if chunk_range is not None:
        return result, counter, (padded, border, L_pad)
    est = ops.ola_finalize(result, counter, border if padded else 0)
    return est.reshape(ni, n_ch, L)


def demucs_chunk_plan(L, chunk_size, num_overlap):
    """Chunk list of utils.demix demucs mode (utils.py:371-375, :408-420): starts 0, step, ...
    while < L, no border pad; returns [(start, seg_len)]."""
    step = chunk_size // num_overlap
    return [(i, min(chunk_size, L - i)) for i in range(0, L, step)]


def demix_device_demucs(config, model, mix, device, exec_batch=None):
    """utils.demix demucs mode (utils.py:371-380, :408-445; taken for model_type 'htdemucs'):
    C = training.samplerate * training.segment, step = C // num_overlap, no fades and no border
    pad, every chunk zero-padded to C, result += y[:seg], counter += 1, then result / counter with
    nan_to_num.  The reference's batch grouping does not change the result here (no per-batch
    window), so chunks run in groups of ``exec_batch``.  Returns the device tensor [n_instr, 2, L]."""
    C = int(config.training.samplerate * config.training.segment)
    ov = int(config.inference.num_overlap)
    ni = len(config.training.instruments)
    if isinstance(mix, torch.Tensor):
        mix_d = mix.to(device=device, dtype=torch.float32).contiguous()
    else:
        mix_d = torch.from_numpy(np.ascontiguousarray(mix, dtype=np.float32)).to(device, non_blocking=False)
    n_ch, L = mix_d.shape
    if L == 0:
        return torch.zeros(ni, n_ch, 0, device=device, dtype=torch.float32)
    plan = demucs_chunk_plan(L, C, ov)
    E = exec_batch or getattr(model, "exec_batch", None) or plan_exec_batch(model, len(plan), C, device)
    ones = torch.ones(C, device=device, dtype=torch.float32)
    result = torch.zeros(ni * n_ch, L, device=device, dtype=torch.float32)
    counter = torch.zeros(L, device=device, dtype=torch.float32)
    xbuf = None
    for pos in range(0, len(plan), E):
        group = plan[pos:pos + E]
        if xbuf is None or xbuf.shape[0] != len(group):
            xbuf = torch.empty(len(group), n_ch, C, device=device, dtype=torch.float32)
        ops.chunk_gather_constant(mix_d, [g[0] for g in group], C, out=xbuf)
        y = model(xbuf).reshape(len(group), ni * n_ch, C)
        ops.ola_accumulate(y, [g[0] for g in group], [g[1] for g in group], ones, result, counter)
    return ops.ola_finalize(result, counter, 0).reshape(ni, n_ch, L)


def demix_pytorch_optimized(config, backend, mix, device, pbar=False):
    """inference_pytorch.demix_pytorch_optimized (:55-186): same signature and return value."""
    dev = torch.device(device) if not isinstance(device, torch.device) else device
    instruments = prefer_target_instrument(config)
    est = demix_device(config, backend, mix, dev, progress=True)
    print("[SESA_PROGRESS]100", flush=True)
    est = est.cpu().numpy()
    return {k: v for k, v in zip(instruments, est)}
