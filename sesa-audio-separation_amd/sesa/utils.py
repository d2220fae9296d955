"""Reference ``utils.py`` surface on the MI355X path.

* ``load_config`` / ``get_model_from_config`` -- utils.py:26-161 (same model_type strings; the
  types without a native implementation raise NotImplementedError naming what exists).
* ``normalize_audio`` / ``denormalize_audio`` -- utils.py:199-238.
* ``demix`` -- utils.py:330-477 (generic mode on the device loop of sesa/demix.py).
* ``apply_tta`` -- utils.py:241-292.
* ``prefer_target_instrument`` -- utils.py:480-499.
* ``load_start_checkpoint`` -- utils.py:585-613 / inference_pytorch.py:326-369 (safe loader).
"""
import numpy as np
import torch

from .config import ConfigDict, load_config, prefer_target_instrument  # noqa: F401
from .demix import demix_device, windowing_array as _getWindowingArray  # noqa: F401

# model_type strings accepted by the reference registry (utils.py:89-157)
REFERENCE_MODEL_TYPES = (
    "mdx23c", "htdemucs", "segm_models", "torchseg", "mel_band_roformer", "bs_roformer", "swin_upernet", "bandit",
    "bandit_v2", "scnet_unofficial", "scnet", "apollo", "bs_mamba2", "experimental_mdx23c_stht",
    "mel_band_roformer_experimental", "bs_roformer_experimental", "bs_roformer_custom", "scnet_tran", "scnet_masked",
    "conformer", "mel_band_conformer")
NATIVE_MODEL_TYPES = ("mdx23c", "htdemucs", "bs_roformer", "mel_band_roformer", "scnet")


def get_model_from_config(model_type: str, config_path: str):
    """utils.get_model_from_config: model_type string -> (model, config)."""
    config = load_config(model_type, config_path)
    if model_type == "mdx23c":
        from .models.mdx23c import TFC_TDF_net
        model = TFC_TDF_net(config)
    elif model_type == "mel_band_roformer":
        from .models.mel_band_roformer import MelBandRoformer
        model = MelBandRoformer(**dict(config.model))  # utils.py:101-103
    elif model_type == "bs_roformer":
        from .models.bs_roformer import BSRoformer
        model = BSRoformer(**dict(config.model))  # utils.py:104-106
    elif model_type == "scnet":
        from .models.scnet import SCNet
        model = SCNet(**dict(config.model))  # utils.py:119-121
    elif model_type == "htdemucs":
        from .models.htdemucs import get_model
        model = get_model(config)  # utils.py:92-94 -> models/demucs4ht.py:696-711
    elif model_type in REFERENCE_MODEL_TYPES:
        raise NotImplementedError(f"model_type '{model_type}' has no MI355X-native implementation yet "
                                  f"(native: {', '.join(NATIVE_MODEL_TYPES)})")
    else:
        raise ValueError(f"Unknown model type: {model_type}")
    return model, config


def normalize_audio(audio: np.ndarray):
    mono = audio.mean(0)
    mean, std = mono.mean(), mono.std()
    return (audio - mean) / std, {"mean": mean, "std": std}


def denormalize_audio(audio: np.ndarray, norm_params):
    return audio * norm_params["std"] + norm_params["mean"]


def _as_backend(model, device):
    """The reference passes either a backend or the raw model to demix / apply_tta
    (inference_pytorch.py:229, :238).  A native model is already a device callable: it is used as
    is, so its precision (set by the session that owns it) is never changed here."""
    return model


def demix(config, model, mix, device, model_type: str = "generic", pbar: bool = False):
    """utils.demix (utils.py:330-477).  Generic mode: the device chunker with fades and border pad.
    model_type 'htdemucs' selects the reference's demucs mode (C = samplerate * segment, no fades,
    no border pad, zero-padded tails, counter += 1) and returns a bare array when the config has
    a single instrument, a dict otherwise (:471-477); the native HTDemucs runs under it."""
    dev = torch.device(device) if not isinstance(device, torch.device) else device
    if model_type == "htdemucs":
        from .demix import demix_device_demucs
        est = demix_device_demucs(config, _as_backend(model, dev), mix, dev).cpu().numpy()
        instruments = list(config.training.instruments)
        if len(instruments) <= 1:
            return est
        return {k: v for k, v in zip(instruments, est)}
    est = demix_device(config, _as_backend(model, dev), mix, dev, progress=False).cpu().numpy()
    return {k: v for k, v in zip(prefer_target_instrument(config), est)}


def apply_tta(config, model, mix, waveforms_orig, device, model_type):
    """utils.apply_tta (:241-292): channel swap + polarity flip, averaged with the original."""
    track_proc_list = [mix[::-1].copy(), -1.0 * mix.copy()]
    for i, augmented_mix in enumerate(track_proc_list):
        waveforms = demix(config, model, augmented_mix, device, model_type=model_type)
        for el in waveforms:
            if i == 0:
                waveforms_orig[el] += waveforms[el][::-1].copy()
            else:
                waveforms_orig[el] -= waveforms[el]
    for el in waveforms_orig:
        waveforms_orig[el] /= len(track_proc_list) + 1
    return waveforms_orig


def load_checkpoint_state(path, map_location="cpu"):
    """Checkpoint -> state_dict (inference_pytorch.py:326-366), with the SAFE loader only
    (weights_only=True): checkpoints that need arbitrary unpickling are refused."""
    ckpt = torch.load(path, map_location=map_location, weights_only=True)
    if isinstance(ckpt, dict):
        for key in ("state_dict", "model", "state"):
            if key in ckpt:
                return ckpt[key]
    return ckpt


def load_start_checkpoint(args, model, type_="inference"):
    """utils.load_start_checkpoint (strict load)."""
    model.load_state_dict(load_checkpoint_state(args.start_check_point), strict=True)
