"""Chunker + windowed overlap-add restatement.  TEST INFRASTRUCTURE.

Restates ``inference_pytorch.demix_pytorch_optimized`` (/root/reference/inference_pytorch.py:55-186),
which is identical in generic mode to ``utils.demix`` (utils.py:330-477), with
every quirk kept:

* fade = C//10, step = C//num_overlap, border = C-step                    (:89-91)
* window = linspace fades (torch.linspace float32)                       (:95-99)
* reflect-pad by ``border`` iff L > 2*border and border > 0               (:102-103)
* chunk i..i+C, padded to C with reflect if len > C//2 else zeros        (:123-138)
* flush when len(batch) >= inference.batch_size or i >= L_pad             (:145)
* window for the WHOLE batch: no fade-in if the last appended chunk starts
  at 0 (``i - step == 0``), elif final batch: no fade-out                 (:151-155)
* result/counter fp32, accumulated in chunk order                        (:157-159)
* est = result / counter, NaN -> 0, crop border                          (:174-180)

Also ``demix_demucs_mode`` restates utils.demix's demucs mode (utils.py:371-380, :420, :444-445)
and ``normalize_audio``/``denormalize_audio`` (utils.py:199-238).
"""
import numpy as np
import torch


def windowing_array(chunk_size, fade_size):
    """utils._getWindowingArray (utils.py:295-327) == inference_pytorch.py:95-99."""
    w = torch.ones(chunk_size)
    w[-fade_size:] = torch.linspace(1, 0, fade_size)
    w[:fade_size] = torch.linspace(0, 1, fade_size)
    return w.numpy()


def chunk_plan(L, chunk_size, num_overlap, batch_size):
    """Return (padded, border, L_pad, batches) where batches = list of (chunks, fade_in_off, fade_out_off)
    and chunks = list of (start, seg_len).  Pure restatement of the loop control at :115-163."""
    step = chunk_size // num_overlap
    border = chunk_size - step
    padded = L > 2 * border and border > 0
    L_pad = L + 2 * border if padded else L
    batches, cur = [], []
    i = 0
    while i < L_pad:
        seg = min(chunk_size, L_pad - i)
        cur.append((i, seg))
        i += step
        if len(cur) >= batch_size or i >= L_pad:
            no_in = (i - step == 0)
            no_out = (not no_in) and i >= L_pad
            batches.append((list(cur), no_in, no_out))
            cur = []
    return padded, border, L_pad, batches


def extract_chunk(mix_pad, start, chunk_size):
    part = mix_pad[:, start:start + chunk_size]
    n = part.shape[-1]
    if n < chunk_size:
        mode = "reflect" if n > chunk_size // 2 else "constant"
        part = np.pad(part, ((0, 0), (0, chunk_size - n)), mode=mode)
    return part


def demix(cfg, model, mix, batch_size=None, num_instruments=None, instruments=None, on_batch=None):
    """demix_pytorch_optimized restated; ``model`` maps torch [B,2,C] f32 -> [B,(n,)2,C]."""
    C = cfg["audio"]["chunk_size"]
    ov = cfg["inference"]["num_overlap"]
    bs = batch_size if batch_size is not None else cfg["inference"]["batch_size"]
    if instruments is None:
        t = cfg["training"].get("target_instrument")
        instruments = [t] if t else list(cfg["training"]["instruments"])
    ni = len(instruments)
    mix = np.asarray(mix, np.float32)
    L = mix.shape[-1]
    fade = C // 10
    win = windowing_array(C, fade)
    padded, border, L_pad, batches = chunk_plan(L, C, ov, bs)
    mix_pad = np.pad(mix, ((0, 0), (border, border)), mode="reflect") if padded else mix
    result = np.zeros((ni, 2, L_pad), np.float32)
    counter = np.zeros((ni, 2, L_pad), np.float32)
    for chunks, no_in, no_out in batches:
        arr = np.stack([extract_chunk(mix_pad, s, C) for s, _ in chunks])
        y = model(torch.from_numpy(arr))
        y = y.detach().cpu().numpy().astype(np.float32)
        if on_batch is not None:
            on_batch(chunks, y)
        w = win.copy()
        if no_in:
            w[:fade] = 1
        elif no_out:
            w[-fade:] = 1
        for j, (s, n) in enumerate(chunks):
            yj = y[j].reshape(ni, 2, C)   # [2,C] broadcasts over a single instrument (:158)
            result[..., s:s + n] += yj[..., :n] * w[:n]
            counter[..., s:s + n] += w[:n]
    with np.errstate(divide="ignore", invalid="ignore"):
        est = result / counter
    np.nan_to_num(est, copy=False, nan=0.0)
    if padded:
        est = est[..., border:-border]
    return {k: v for k, v in zip(instruments, est)}


def demix_demucs_mode(cfg, model, mix):
    """utils.demix with model_type 'htdemucs' (utils.py:371-380, :408-445, :471-477) restated:
    C = training.samplerate * training.segment, step = C // num_overlap, no border pad and no
    fades; chunk i..i+C zero-padded to C ('constant' whatever its length, :413-418); batches of
    inference.batch_size; result += y[:seg], counter += 1.0 in chunk order; result / counter,
    NaN -> 0.  Returns the bare array for a single instrument, else {instrument: [2, L]}."""
    C = int(cfg["training"]["samplerate"] * cfg["training"]["segment"])
    step = C // cfg["inference"]["num_overlap"]
    bs = cfg["inference"]["batch_size"]
    instruments = list(cfg["training"]["instruments"])
    ni = len(instruments)
    mix = np.asarray(mix, np.float32)
    L = mix.shape[-1]
    result = np.zeros((ni,) + mix.shape, np.float32)
    counter = np.zeros((ni,) + mix.shape, np.float32)
    i, batch, locs = 0, [], []
    while i < L:
        part = mix[:, i:i + C]
        n = part.shape[-1]
        batch.append(np.pad(part, ((0, 0), (0, C - n))))
        locs.append((i, n))
        i += step
        if len(batch) >= bs or i >= L:
            y = model(torch.from_numpy(np.stack(batch))).detach().cpu().numpy().astype(np.float32)
            for j, (s, n) in enumerate(locs):
                result[..., s:s + n] += y[j, ..., :n]
                counter[..., s:s + n] += 1.0
            batch, locs = [], []
    with np.errstate(divide="ignore", invalid="ignore"):
        est = result / counter
    np.nan_to_num(est, copy=False, nan=0.0)
    if ni <= 1:
        return est
    return {k: v for k, v in zip(instruments, est)}


def normalize_audio(audio):
    """utils.normalize_audio (utils.py:199-217)."""
    mono = audio.mean(0)
    mean, std = mono.mean(), mono.std()
    return (audio - mean) / std, {"mean": mean, "std": std}


def denormalize_audio(audio, p):
    """utils.denormalize_audio (utils.py:220-238)."""
    return audio * p["std"] + p["mean"]
