"""CLI drop-in for ``inference.py`` / ``inference_pytorch.py`` of the reference.

Same flags (inference.py:159-181, inference_pytorch.py:281-303), same per-file flow
(inference_pytorch.py:189-274): read -> (normalize) -> demix -> (TTA) -> (demud phase remix) ->
(extract instrumental) -> (denormalize) -> write ``<short(name)>_<instr>.<ext>`` into --store_dir,
``[SESA_PROGRESS]N`` lines on stdout, non-zero exit on failure.

Differences (all deliberate, all loud):
* the device is a HIP GPU; ``--force_cpu`` is rejected (there is no CPU path);
* checkpoints load with ``torch.load(weights_only=True)`` only;
* audio I/O is sesa/audio_io.py: WAV and FLAC (libsesa's FLAC codec); mp3 / ogg / m4a inputs have
  no offline decoder and are skipped with the reference's "cannot read track" message;
* ``--lora_checkpoint`` is accepted and ignored (LoRA is not on the inference path).

Run:  python -m sesa.inference --model_type mdx23c --config_path C.yaml --start_check_point W.ckpt \
          --input_folder in/ --store_dir out/
"""
import argparse
import glob
import os
import sys
import time

import numpy as np
import torch


def shorten_filename(filename, max_length=30):
    """inference_pytorch.shorten_filename (:34-40)."""
    base, ext = os.path.splitext(filename)
    if len(base) <= max_length:
        return filename
    return base[:15] + "..." + base[-10:] + ext


def get_soundfile_subtype(pcm_type, is_float=False):
    """inference_pytorch.get_soundfile_subtype (:43-52)."""
    if is_float:
        return "FLOAT"
    return {"PCM_16": "PCM_16", "PCM_24": "PCM_24", "FLOAT": "FLOAT"}.get(pcm_type, "FLOAT")


def build_parser():
    p = argparse.ArgumentParser(description="MI355X Inference for Music Source Separation")
    p.add_argument("--model_type", type=str, default="mdx23c")
    p.add_argument("--config_path", type=str)
    p.add_argument("--start_check_point", type=str, default="")
    p.add_argument("--input_folder", type=str)
    p.add_argument("--audio_path", type=str, default="")
    p.add_argument("--store_dir", type=str, default="")
    p.add_argument("--device_ids", nargs="+", type=int, default=0)
    p.add_argument("--extract_instrumental", action="store_true")
    p.add_argument("--disable_detailed_pbar", action="store_true")
    p.add_argument("--force_cpu", action="store_true")
    p.add_argument("--flac_file", action="store_true")
    p.add_argument("--export_format", type=str, choices=["wav FLOAT", "flac PCM_16", "flac PCM_24"],
                   default="flac PCM_24")
    p.add_argument("--pcm_type", type=str, choices=["PCM_16", "PCM_24"], default="PCM_24")
    p.add_argument("--chunk_size", type=int, default=1000000)   # parsed but unused, as in the reference
    p.add_argument("--overlap", type=int, default=4)             # parsed but unused, as in the reference
    p.add_argument("--optimize_mode", type=str, choices=["channels_last", "compile", "jit", "default"],
                   default="channels_last")
    p.add_argument("--enable_amp", action="store_true", help="throughput precision: MDX23C fp16 TFC convs (~5e-5 RMS), others single-pass bf16")
    p.add_argument("--enable_tf32", action="store_true")
    p.add_argument("--enable_cudnn_benchmark", action="store_true")
    p.add_argument("--lora_checkpoint", type=str, default="")
    p.add_argument("--use_tta", action="store_true")
    p.add_argument("--demud_phaseremix_inst", action="store_true")
    p.add_argument("--exec_batch", type=int, default=0,
                   help="chunks per native forward (MI355X only; 0 = planned from the model and free HBM)")
    return p


def run_folder(backend, model, args, config, device):
    from .audio_io import read_audio, write_audio
    from .config import prefer_target_instrument
    from .demix import demix_pytorch_optimized
    from .utils import apply_tta, demix, denormalize_audio, normalize_audio

    start = time.time()
    if args.audio_path:
        paths = [args.audio_path]
    else:
        paths = sorted(glob.glob(os.path.join(args.input_folder, "*.*")))
    sr = getattr(config.audio, "sample_rate", 44100)
    print(f"MI355X backend | {len(paths)} files | SR: {sr}")
    instruments = prefer_target_instrument(config)[:]
    os.makedirs(args.store_dir, exist_ok=True)
    for path in paths:
        try:
            mix, sr_ = read_audio(path, sr=sr)
        except Exception as e:
            print(f"Cannot read track: {path}\nError: {e}")
            continue
        if mix.shape[0] == 1:
            mix = np.concatenate([mix, mix], 0)   # reference would fail on mono (1-D librosa output)
        mix_orig = mix.copy()
        norm = None
        if "normalize" in config.inference and config.inference["normalize"] is True:
            mix, norm = normalize_audio(mix)
        wav = demix_pytorch_optimized(config, backend, mix, device, pbar=not args.disable_detailed_pbar)
        if args.use_tta:
            wav = apply_tta(config, backend, mix, wav, device, args.model_type)
        if args.demud_phaseremix_inst:
            instr = "vocals" if "vocals" in instruments else instruments[0]
            instruments.append("instrumental_phaseremix")
            if "instrumental" not in instruments and "Instrumental" not in instruments:
                mod = mix_orig - 2 * wav[instr]
                wm = demix(config, backend, mod, device, model_type=args.model_type)
                if args.use_tta:
                    wm = apply_tta(config, backend, mod, wm, device, args.model_type)
                wav["instrumental_phaseremix"] = mix_orig + wm[instr]
            else:
                mod = 2 * wav[instr] - mix_orig
                mod_ = mod.copy()
                wm = demix(config, backend, mod, device, model_type=args.model_type)
                if args.use_tta:
                    wm = apply_tta(config, backend, mod, wav, device, args.model_type)
                wav["instrumental_phaseremix"] = mix_orig + mod_ - wm[instr]
        if args.extract_instrumental:
            instr = "vocals" if "vocals" in instruments else instruments[0]
            wav["instrumental"] = mix_orig - wav[instr]
            if "instrumental" not in instruments:
                instruments.append("instrumental")
        for instr in instruments:
            est = wav[instr]
            if norm is not None:
                est = denormalize_audio(est, norm)
            is_float = getattr(args, "export_format", "").startswith("wav FLOAT")   # :262-272
            codec = "flac" if getattr(args, "flac_file", False) else "wav"
            subtype = get_soundfile_subtype(args.pcm_type if codec == "flac" else "FLOAT", is_float)
            out = os.path.join(args.store_dir, f"{shorten_filename(os.path.basename(path))}_{instr}.{codec}")
            write_audio(out, est.T, sr, subtype=subtype)
    print(f"Elapsed time: {time.time() - start:.2f} sec")


def proc_folder(argv=None):
    args = build_parser().parse_args(argv)
    if args.force_cpu:
        print("ERROR: --force_cpu is not supported: the MI355X path has no CPU fallback", file=sys.stderr)
        return 2
    if not torch.cuda.is_available():
        print("ERROR: no HIP device visible", file=sys.stderr)
        return 2
    ids = args.device_ids if isinstance(args.device_ids, list) else [args.device_ids]
    device = f"cuda:{ids[0]}"
    torch.cuda.set_device(ids[0])
    from .backend import create_inference_session
    from .utils import get_model_from_config, load_checkpoint_state
    t0 = time.time()
    model, config = get_model_from_config(args.model_type, args.config_path)
    if args.start_check_point:
        try:
            sd = load_checkpoint_state(args.start_check_point)
        except Exception as e:
            print(f"CHECKPOINT FILE CORRUPTED OR UNSAFE\nError: {e}\nFile: {args.start_check_point}")
            return 1
        model.load_state_dict(sd, strict=False)   # inference_pytorch.py:368
    print(f"Instruments: {config.training.instruments}")
    backend = create_inference_session(model, device=device, optimize_mode=args.optimize_mode,
                                       enable_amp=args.enable_amp, enable_tf32=args.enable_tf32,
                                       enable_cudnn_benchmark=args.enable_cudnn_benchmark,
                                       exec_batch=args.exec_batch or None)
    print(f"Model load time: {time.time() - t0:.2f} sec")
    run_folder(backend, model, args, config, device)
    return 0


if __name__ == "__main__":
    sys.exit(proc_folder())
