"""ctypes binding of libsesa (include/sesa.h).  The product path has NO fallback: if the HIP
library is missing or no HIP device is usable, importing/using these entry points raises."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SESA_LIB", os.path.join(_HERE, "_native", "libsesa.so"))

c_int, c_int64, c_size_t, c_void_p, c_char_p = ctypes.c_int, ctypes.c_int64, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_char_p
P_f32 = ctypes.c_void_p
P_i64 = ctypes.POINTER(ctypes.c_int64)

SESA_PREC_BF16X3 = 0
SESA_PREC_BF16 = 1
SESA_PREC_F16W2 = 2
SESA_PREC_F16 = 3
SESA_PREC_F16MIX = 4


class SesaMdx23cConfig(ctypes.Structure):
    _fields_ = [(n, c_int) for n in (
        "chunk_size", "dim_f", "dim_t", "hop_length", "n_fft", "audio_channels",
        "num_subbands", "num_scales", "num_blocks_per_scale", "num_channels",
        "growth", "bottleneck_factor", "scale_t", "scale_f", "num_instruments", "precision")]


class SesaBsrConfig(ctypes.Structure):
    _fields_ = [(n, c_int) for n in (
        "chunk_size", "audio_channels", "n_fft", "hop_length", "win_length", "dim", "depth", "heads", "dim_head",
        "time_transformer_depth", "freq_transformer_depth", "num_stems", "mask_estimator_depth",
        "mlp_expansion_factor", "n_bands")] + [("freqs_per_bands", ctypes.POINTER(c_int)), ("precision", c_int),
                                               ("mel", c_int), ("n_freq_indices", c_int),
                                               ("freq_indices", ctypes.POINTER(c_int))]


class SesaScnetConfig(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("chunk_size", "audio_channels", "n_sources", "n_fft", "hop_size", "win_size",
                                     "normalized", "n_dims")] + [
        ("dims", ctypes.POINTER(c_int)), ("band_sr", ctypes.c_double * 3), ("band_stride", c_int * 3),
        ("band_kernel", c_int * 3), ("conv_depths", c_int * 3), ("compress", c_int), ("conv_kernel", c_int),
        ("num_dplayer", c_int), ("expand", c_int), ("precision", c_int)]


class SesaHtdemucsConfig(ctypes.Structure):
    _fields_ = [(n, c_int) for n in (
        "chunk_size", "audio_channels", "n_sources", "channels", "channels_time", "growth", "nfft", "depth",
        "kernel_size", "stride", "context", "context_enc", "norm_starts", "rewrite", "cac", "num_subbands",
        "dconv_mode", "dconv_depth", "dconv_comp", "bottom_channels", "t_layers", "t_heads", "t_norm_in",
        "t_norm_first", "t_norm_out", "t_layer_scale", "t_gelu", "t_cross_first")] + [
        (n, ctypes.c_double) for n in ("t_hidden_scale", "freq_emb", "emb_scale", "t_max_period",
                                       "t_weight_pos_embed")] + [("precision", c_int)]


# name -> (restype, argtypes); every symbol declared in include/sesa.h
SIGNATURES = {
    "sesa_version": (c_int, []),
    "sesa_last_error": (c_char_p, []),
    "sesa_stft_f32": (c_int, [P_f32, c_int, c_int, c_int, c_int, c_int, P_f32, c_void_p]),
    "sesa_istft_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "sesa_istft_f32": (c_int, [P_f32, c_int, c_int, c_int, c_int, c_int, P_f32, c_void_p, c_void_p]),
    "sesa_chunk_gather_f32": (c_int, [P_f32, c_int, c_int64, c_int64, P_i64, c_int, c_int, P_f32, c_void_p]),
    "sesa_chunk_gather_constant_f32": (c_int, [P_f32, c_int, c_int64, P_i64, c_int, c_int, P_f32, c_void_p]),
    "sesa_ola_accumulate_f32": (c_int, [P_f32, c_int, c_int, c_int, P_i64, P_i64, P_f32, P_f32, P_f32, c_int64,
                                        c_void_p]),
    "sesa_ola_finalize_f32": (c_int, [P_f32, P_f32, c_int, c_int64, c_int64, P_f32, c_void_p]),
    "sesa_mdx23c_create": (c_int, [ctypes.POINTER(SesaMdx23cConfig), ctypes.POINTER(c_void_p)]),
    "sesa_mdx23c_num_params": (c_int, [c_void_p]),
    "sesa_mdx23c_param_info": (c_int, [c_void_p, c_int, ctypes.POINTER(c_char_p), ctypes.POINTER(c_int64)]),
    "sesa_mdx23c_set_param": (c_int, [c_void_p, c_char_p, P_f32, c_int64]),
    "sesa_mdx23c_finalize": (c_int, [c_void_p, c_void_p]),
    "sesa_mdx23c_workspace_size": (c_size_t, [c_void_p, c_int]),
    "sesa_mdx23c_forward": (c_int, [c_void_p, P_f32, c_int, P_f32, c_void_p, c_size_t, c_void_p]),
    "sesa_mdx23c_destroy": (c_int, [c_void_p]),
    "sesa_mdx23c_set_conv_variant": (c_int, [c_int]),
    "sesa_mdx23c_set_wino": (c_int, [c_int]),
    "sesa_mdx23c_set_f16_plan": (c_int, [c_char_p, c_char_p]),
    "sesa_mdx23c_set_tdf_plan": (c_int, [c_char_p, c_char_p]),
    "sesa_bsr_create": (c_int, [ctypes.POINTER(SesaBsrConfig), ctypes.POINTER(c_void_p)]),
    "sesa_bsr_num_params": (c_int, [c_void_p]),
    "sesa_bsr_param_info": (c_int, [c_void_p, c_int, ctypes.POINTER(c_char_p), ctypes.POINTER(c_int64)]),
    "sesa_bsr_set_param": (c_int, [c_void_p, c_char_p, P_f32, c_int64]),
    "sesa_bsr_finalize": (c_int, [c_void_p, c_void_p]),
    "sesa_bsr_workspace_size": (c_size_t, [c_void_p, c_int]),
    "sesa_bsr_forward": (c_int, [c_void_p, P_f32, c_int, P_f32, c_void_p, c_size_t, c_void_p]),
    "sesa_bsr_destroy": (c_int, [c_void_p]),
    "sesa_scnet_create": (c_int, [ctypes.POINTER(SesaScnetConfig), ctypes.POINTER(c_void_p)]),
    "sesa_scnet_num_params": (c_int, [c_void_p]),
    "sesa_scnet_param_info": (c_int, [c_void_p, c_int, ctypes.POINTER(c_char_p), ctypes.POINTER(c_int64)]),
    "sesa_scnet_set_param": (c_int, [c_void_p, c_char_p, P_f32, c_int64]),
    "sesa_scnet_finalize": (c_int, [c_void_p, c_void_p]),
    "sesa_scnet_workspace_size": (c_size_t, [c_void_p, c_int]),
    "sesa_scnet_forward": (c_int, [c_void_p, P_f32, c_int, P_f32, c_void_p, c_size_t, c_void_p]),
    "sesa_scnet_destroy": (c_int, [c_void_p]),
    "sesa_htdemucs_create": (c_int, [ctypes.POINTER(SesaHtdemucsConfig), ctypes.POINTER(c_void_p)]),
    "sesa_htdemucs_num_params": (c_int, [c_void_p]),
    "sesa_htdemucs_param_info": (c_int, [c_void_p, c_int, ctypes.POINTER(c_char_p), ctypes.POINTER(c_int64)]),
    "sesa_htdemucs_param_shape": (c_int, [c_void_p, c_int, ctypes.POINTER(c_int64), ctypes.POINTER(c_int)]),
    "sesa_htdemucs_set_param": (c_int, [c_void_p, c_char_p, P_f32, c_int64]),
    "sesa_htdemucs_finalize": (c_int, [c_void_p, c_void_p]),
    "sesa_htdemucs_workspace_size": (c_size_t, [c_void_p, c_int]),
    "sesa_htdemucs_forward": (c_int, [c_void_p, P_f32, c_int, P_f32, c_void_p, c_size_t, c_void_p]),
    "sesa_htdemucs_destroy": (c_int, [c_void_p]),
    "sesa_blend_workspace_size": (c_size_t, [c_int, c_int64]),
    "sesa_blend_workspace_size_n": (c_size_t, [c_int, c_int, c_int64]),
    "sesa_blend_f32": (c_int, [P_f32, c_int, c_int, c_int64, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_size_t,
                               c_void_p]),
    "sesa_flac_info": (c_int, [c_void_p, c_size_t, ctypes.POINTER(c_int), ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                               ctypes.POINTER(c_int64)]),
    "sesa_flac_decode": (c_int, [c_void_p, c_size_t, c_void_p, c_int64, ctypes.POINTER(c_int64)]),
    "sesa_flac_encode_bound": (c_size_t, [c_int64, c_int, c_int]),
    "sesa_flac_encode": (c_int, [c_void_p, c_int64, c_int, c_int, c_int, c_void_p, c_size_t, ctypes.POINTER(c_size_t)]),
    "sesa_profile_enable": (c_int, [c_int]),
    "sesa_profile_read": (c_int, [c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_int64),
                                  ctypes.POINTER(ctypes.c_double)]),
    "sesa_profile_read2": (c_int, [c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_int64),
                                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "sesa_profile_floor": (c_int, [c_int, ctypes.c_double, ctypes.c_double, ctypes.POINTER(ctypes.c_double)]),
    "sesa_debug_trace_begin": (c_int, [c_void_p, c_int]),
    "sesa_debug_trace_end": (c_int, [ctypes.POINTER(c_int), c_int]),
}

KCLASS = {"conv3x3": 0, "conv1x1": 1, "down": 2, "up": 3, "tdf": 4, "stft": 5, "istft": 6, "act": 7, "tokgemm": 8,
          "attn": 9, "lstm": 10, "simt": 11, "ola": 12, "hconv": 13, "conv3x3_x3": 14, "dft": 15}


def profile_enable(on):
    check(lib().sesa_profile_enable(1 if on else 0), "sesa_profile_enable")


def profile_read(kclass):
    ms, n, work = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
    check(lib().sesa_profile_read(KCLASS[kclass] if isinstance(kclass, str) else kclass, ctypes.byref(ms),
                                  ctypes.byref(n), ctypes.byref(work)), "sesa_profile_read")
    return ms.value, n.value, work.value


def profile_read2(kclass):
    """(ms, launches, algorithmic work, algorithmic HBM bytes) of a kernel class (sesa_profile_read2)."""
    ms, n, work, nb = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
    check(lib().sesa_profile_read2(KCLASS[kclass] if isinstance(kclass, str) else kclass, ctypes.byref(ms),
                                   ctypes.byref(n), ctypes.byref(work), ctypes.byref(nb)), "sesa_profile_read2")
    return ms.value, n.value, work.value, nb.value


def profile_floor(kclass, peak_tflops, peak_gbs):
    """Sum over the class's launches of max(FLOP / peak, bytes / HBM peak), ms (sesa_profile_floor)."""
    f = ctypes.c_double()
    check(lib().sesa_profile_floor(KCLASS[kclass] if isinstance(kclass, str) else kclass, float(peak_tflops),
                                   float(peak_gbs), ctypes.byref(f)), "sesa_profile_floor")
    return f.value


class SesaError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libsesa.so (once).  Raises ImportError if the HIP library was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libsesa not built: {LIB_PATH} missing (run __graft_entry__.build() or "
                              f"`make -C sesa-audio-separation_amd/csrc`)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, what=""):
    if rc != 0:
        msg = lib().sesa_last_error()
        raise SesaError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
    return rc


def i64_array(values):
    arr = (ctypes.c_int64 * len(values))(*[int(v) for v in values])
    return arr
