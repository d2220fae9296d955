"""Ensemble blend on the MI355X path -- drop-in for ``/root/reference/ensemble.py``.

Same CLI (``--files ... --type {avg_wave,median_wave,max_wave,min_wave,max_fft,min_fft,median_fft}
[--weights ...] --output P [--buffer 32768]``, exit 0/1, :409-438), same ``[SESA_PROGRESS]N`` lines,
same validation rules (stereo, >= 2 files, one sample rate, :86-170), inputs cut to the shortest
(:304-306), output written as 2-channel PCM_24 WAV (:311).  The blend itself -- every buffer of
every method, including the scipy-STFT magnitude methods -- runs in libsesa ``sesa_blend_f32``
(csrc/sesa_blend.hip) in float64 on the device; there is no CPU fallback.

Divergence kept from the reference on purpose: the path-sanitising re-encode (:63-84), which
re-writes inputs whose path contains one of ``[]()|&; `` as PCM_16 through librosa, is
reproduced only as the quantisation it causes (``requantize_special_paths=True``, default).
"""
import argparse
import os
import sys
import warnings

import numpy as np
import torch

from . import _native as N
from .audio_io import quantize_pcm, read_wav, write_audio

METHODS = ["avg_wave", "median_wave", "max_wave", "min_wave", "max_fft", "min_fft", "median_fft"]
# Member precisions of the configs[4] ensemble line (bench.py --model ensemble) and of its parity gate
# (tests/test_ensemble_models.py: every blend method within 8e-5 of the reference on three fixtures).  The
# spectral blends take the phase of file 0 -- the MDX23C stem -- and a magnitude from another member, so they
# multiply MDX23C's relative error by that member's magnitude over MDX23C's in every bin: measured on MI355X
# (tools/ens_parity_scan.py, profiles/r05_ens_parity_scan.txt) max_fft reaches 9.5e-4 and median_fft 1.4e-4 with
# the MDX23C member in fp16mix (and 5.6e-4 / 1.3e-4 with only its level 0-1 convs in bf16x3), 4.1e-5 / 8.8e-6 with
# it in bf16x3; BS-Roformer fp16 and SCNet fp16mix keep every blend within 4.1e-5.
ENSEMBLE_PRECISIONS = {"mdx23c": "bf16x3", "bs_roformer": "fp16", "scnet": "fp16mix"}
_SPECIAL = "[]()|&; "


def blend_device(waves, method, weights=None, buffer=32768):
    """[n_files, ch, L] (array or device tensor) -> device float64 [ch, L] (run_ensemble's buffer loop)."""
    if method not in METHODS:
        raise ValueError(f"Invalid method '{method}'. Available: {METHODS}")
    x = torch.as_tensor(waves).to("cuda", torch.float32).contiguous()
    if not x.is_cuda:
        raise N.SesaError("blend_device needs a HIP device (no CPU fallback)")
    n, ch, L = x.shape
    out = torch.empty(ch, L, device=x.device, dtype=torch.float64)
    w = None
    if weights is not None and len(weights) == n:
        w = np.ascontiguousarray(np.asarray(weights, np.float32))
    ws_bytes = N.lib().sesa_blend_workspace_size_n(n, ch, int(buffer))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device) if method.endswith("_fft") else None
    N.check(N.lib().sesa_blend_f32(x.data_ptr(), n, ch, L, int(buffer), METHODS.index(method),
                                   w.ctypes.data if w is not None else None, out.data_ptr(),
                                   ws.data_ptr() if ws is not None else None, ws_bytes if ws is not None else 0,
                                   torch.cuda.current_stream(x.device).cuda_stream), "sesa_blend_f32")
    return out


def ensemble_separate(members, mix_d, stem="vocals", method="avg_wave", weights=None, buffer=32768, rank=None,
                      world=None, exec_batch=None, group=None, demix_hooks=None, blend_fn=None, gather_to=0,
                      simulate=False, streams=1):
    """Multi-model ensemble of one track, all on the device (BASELINE configs[4]).

    The GUI's ensemble flow (processing.py:266-363 runs inference.py once per model, then
    ensemble.py blends the chosen stem files) without the per-model WAV round trip: every member
    ``(config, model)`` separates the device-resident mix [2, L] chunk-sharded over the process
    group (sesa/parallel.py: contiguous chunk ranges per rank, one RCCL gather per model to rank
    ``gather_to``), the members' ``stem`` outputs are stacked and blended with ``sesa_blend_f32``
    (ensemble.py:258-407 semantics, float64) on that rank.  Returns (blend [2, L] float64, {member index:
    stem [2, L] float32}) there and (None, {}) on the other ranks (``gather_to=None``: every rank blends).
    ``exec_batch``: chunks per forward, a list (one per member) or an int.  ``streams``: forwards of each member in
    flight on side streams (bit-identical to 1, include/sesa.h).  ``demix_hooks`` (local_fn /
    counter_fn / finalize_fn of demix_sharded) and ``blend_fn`` exist so the CPU test-suite can drive the
    sharding, the collectives and the member loop over gloo ranks with the oracle's OLA and blend."""
    from .config import prefer_target_instrument
    from .parallel import demix_sharded
    stems = []
    restore = _spectral_blend_precisions(members, method)
    try:
        for i, (cfg, model) in enumerate(members):
            names = prefer_target_instrument(cfg)
            if stem not in names:
                raise ValueError(f"ensemble member {i} has no '{stem}' stem (instruments: {names})")
            eb = exec_batch[i] if isinstance(exec_batch, (list, tuple)) else (exec_batch or 8)
            est = demix_sharded(cfg, model, mix_d, mix_d.device, rank=rank, world=world, exec_batch=eb, group=group,
                                gather_to=gather_to, simulate=simulate, streams=streams, **(demix_hooks or {}))
            if est is not None:
                stems.append(est[names.index(stem)])
    finally:
        for model, prec in restore:
            model.set_precision(prec)
    if not stems:
        return None, {}
    x = torch.stack(stems)
    return (blend_fn or blend_device)(x, method, weights, buffer), {i: s for i, s in enumerate(stems)}


def _spectral_blend_precisions(members, method):
    """The spectral blends (max_fft / min_fft / median_fft) take file 0's phase and another member's magnitude per bin,
    so they amplify an MDX23C member's rounding error (fp16mix: 9.5e-4 max_fft on the full-width fixtures against
    4.1e-5 in bf16x3, profiles/r05_ens_parity_scan.txt).  For those methods every MDX23C member not already in bf16x3
    runs bf16x3 for this call (with a warning); returns [(model, precision to restore)]."""
    if not method.endswith("_fft"):
        return []
    restore = []
    for i, (_, model) in enumerate(members):
        m = getattr(model, "module", model)   # nn.DataParallel
        if getattr(m, "_prefix", None) == "mdx23c" and getattr(m, "precision", "bf16x3") != "bf16x3":
            warnings.warn(f"ensemble member {i} (MDX23C, {m.precision}): the {method} blend amplifies its rounding "
                          f"error past the 1e-4 parity gate; running it in bf16x3 for this ensemble")
            restore.append((m, m.precision))
            m.set_precision("bf16x3")
    return restore


class AudioEnsembleEngine:
    """ensemble.AudioEnsembleEngine surface: process_waveform / process_spectral / run_ensemble."""

    def __init__(self, requantize_special_paths=True):
        self.requantize_special_paths = requantize_special_paths

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def process_waveform(self, chunks, method, weights=None):
        return blend_device(chunks, method, weights, buffer=max(1, np.shape(chunks)[-1])).cpu().numpy()

    def process_spectral(self, chunks, method):
        chunks = np.asarray(chunks)
        if chunks.shape[-1] < 256:
            return None
        return blend_device(chunks, method, None, buffer=chunks.shape[-1]).cpu().numpy()

    def _load(self, path):
        data, sr = read_wav(path)                       # float32 [ch, frames], soundfile scaling
        if self.requantize_special_paths and any(c in os.path.abspath(path) for c in _SPECIAL):
            # librosa.load + sf.write(temp) at soundfile's default PCM_16, read back (ensemble.py:70-79):
            # libsndfile's float -> PCM_16 write is lrintf(x * 0x7FFF) (no clipping), its read x / 0x8000
            data = (quantize_pcm(data, 16) / 32768.0).astype(np.float32)
        return data, sr

    def validate_inputs(self, files, method):
        errors, valid, rates, loaded = [], [], set(), []
        if method not in METHODS:
            errors.append(f"Invalid method '{method}'. Available: {METHODS}")
        for f in files:
            if not os.path.exists(f):
                errors.append(f"File not found: {f}")
                continue
            if os.path.getsize(f) == 0:
                errors.append(f"Empty file: {f}")
                continue
            try:
                data, sr = self._load(f)
            except Exception as e:  # noqa: BLE001 -- reported like the reference
                errors.append(f"Invalid audio file {f}: {e}")
                continue
            if data.shape[0] != 2:
                errors.append(f"File must be stereo (has {data.shape[0]} channels): {f}")
                continue
            rates.add(sr)
            valid.append(f)
            loaded.append(data)
        if len(valid) < 2:
            errors.append("At least 2 valid files required")
        if len(rates) > 1:
            errors.append(f"Sample rate mismatch: {rates}")
        if errors:
            raise ValueError("\n".join(errors))
        return valid, loaded, rates.pop()

    def run_ensemble(self, files, method, output_path, weights=None, buffer_size=32768):
        try:
            valid, loaded, sr = self.validate_inputs(files, method)
            out_dir = os.path.dirname(os.path.abspath(output_path)) or "."
            os.makedirs(out_dir, exist_ok=True)
            if weights and len(weights) == len(valid):
                w = np.asarray(weights, np.float32)
            else:
                w = None
            shortest = min(d.shape[1] for d in loaded)
            print("Loading audio files...", flush=True)
            waves = np.stack([d[:, :shortest] for d in loaded])
            print("Processing ensemble...", flush=True)
            out = blend_device(waves, method, w, buffer_size).cpu().numpy()
            total = (shortest + buffer_size - 1) // buffer_size
            last = -1
            for k in range(1, total + 1):                     # progress protocol (:379-383)
                pct = int((k / total) * 100)
                if pct > last:
                    last = pct
                    print(f"[SESA_PROGRESS]{pct}", flush=True)
            print("Saving ensemble output...", flush=True)
            write_audio(output_path, out.T, sr, subtype="PCM_24")
            print(f"\nEnsemble completed successfully: {output_path}")
            return True
        except Exception as e:  # noqa: BLE001 -- the reference turns every failure into exit code 1
            print(f"\nError during processing: {e}", file=sys.stderr)
            return False


def build_parser():
    p = argparse.ArgumentParser(description="Ultimate Audio Ensemble Processor - Supports all ensemble methods",
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument("--files", nargs="+", required=True, help="Input audio files (supports special characters)")
    p.add_argument("--type", required=True, choices=METHODS, help="Ensemble method to use")
    p.add_argument("--weights", nargs="+", type=float, help="Relative weights for each input file")
    p.add_argument("--output", required=True, help="Output file path")
    p.add_argument("--buffer", type=int, default=32768, help="Buffer size in samples (larger=faster but uses more memory)")
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)
    with AudioEnsembleEngine() as engine:
        ok = engine.run_ensemble(files=args.files, method=args.type, output_path=args.output, weights=args.weights,
                                 buffer_size=args.buffer)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
