"""PyTorch-ROCm custom ops over the libsesa C ABI (namespace ``sesa::``).

Each op takes device tensors, launches on the current torch HIP stream *of the tensors' device*
(under that device, so a caller passing ``cuda:1`` without ``set_device`` gets its kernels ordered
after the producers on that device) and returns device tensors; there is no CPU implementation
and no fallback (a CPU tensor is an error).
"""
import contextlib

import torch

from . import _native as N


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _on(t):
    return torch.cuda.device(t.device) if t.is_cuda else contextlib.nullcontext()


def _dev_f32(t, name):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise N.SesaError(f"{name}: expected a HIP device tensor (got {type(t).__name__} "
                          f"on {getattr(t, 'device', None)}); the sesa path has no CPU fallback")
    if t.dtype != torch.float32:
        raise N.SesaError(f"{name}: expected float32, got {t.dtype}")
    return t.contiguous()


@torch.library.custom_op("sesa::stft", mutates_args=())
def stft(x: torch.Tensor, n_fft: int, hop: int, dim_f: int) -> torch.Tensor:
    """models/mdx23c_tfc_tdf_v3.py:14-30 on [..., L] signals -> [..., 2, dim_f, frames]."""
    x = _dev_f32(x, "sesa::stft")
    lead = x.shape[:-1]
    L = x.shape[-1]
    n_sig = 1
    for s in lead:
        n_sig *= int(s)
    frames = 1 + L // hop
    out = torch.empty(*lead, 2, dim_f, frames, device=x.device, dtype=torch.float32)
    with _on(x):
        N.check(N.lib().sesa_stft_f32(x.data_ptr(), n_sig, L, n_fft, hop, dim_f, out.data_ptr(), _stream(x)),
                "sesa_stft_f32")
    return out


@stft.register_fake
def _(x, n_fft, hop, dim_f):
    return x.new_empty(*x.shape[:-1], 2, dim_f, 1 + x.shape[-1] // hop)


@torch.library.custom_op("sesa::istft", mutates_args=())
def istft(spec: torch.Tensor, n_fft: int, hop: int) -> torch.Tensor:
    """models/mdx23c_tfc_tdf_v3.py:32-44 on [..., 2, dim_f, frames] -> [..., hop*(frames-1)]."""
    spec = _dev_f32(spec, "sesa::istft")
    lead = spec.shape[:-3]
    dim_f, frames = spec.shape[-2], spec.shape[-1]
    n_sig = 1
    for s in lead:
        n_sig *= int(s)
    out = torch.empty(*lead, hop * (frames - 1), device=spec.device, dtype=torch.float32)
    ws = torch.empty(N.lib().sesa_istft_workspace_size(n_sig, frames, n_fft) // 4, device=spec.device,
                     dtype=torch.float32)
    with _on(spec):
        N.check(N.lib().sesa_istft_f32(spec.data_ptr(), n_sig, dim_f, frames, n_fft, hop, out.data_ptr(),
                                       ws.data_ptr(), _stream(spec)), "sesa_istft_f32")
    return out


@istft.register_fake
def _(spec, n_fft, hop):
    return spec.new_empty(*spec.shape[:-3], hop * (spec.shape[-1] - 1))


def chunk_gather(mix, border, starts, chunk, out=None):
    """inference_pytorch.py:102-103, :125-138 -> [n_chunks, n_ch, chunk]."""
    mix = _dev_f32(mix, "sesa chunk_gather")
    n_ch, L = mix.shape
    if out is None:
        out = torch.empty(len(starts), n_ch, chunk, device=mix.device, dtype=torch.float32)
    with _on(mix):
        N.check(N.lib().sesa_chunk_gather_f32(mix.data_ptr(), n_ch, L, border, N.i64_array(starts), len(starts),
                                              chunk, out.data_ptr(), _stream(mix)), "sesa_chunk_gather_f32")
    return out


def chunk_gather_constant(mix, starts, chunk, out=None):
    """utils.py:413-418 in demucs mode: no border pad, short chunks zero-padded -> [n_chunks, n_ch, chunk]."""
    mix = _dev_f32(mix, "sesa chunk_gather_constant")
    n_ch, L = mix.shape
    if out is None:
        out = torch.empty(len(starts), n_ch, chunk, device=mix.device, dtype=torch.float32)
    with _on(mix):
        N.check(N.lib().sesa_chunk_gather_constant_f32(mix.data_ptr(), n_ch, L, N.i64_array(starts), len(starts),
                                                       chunk, out.data_ptr(), _stream(mix)),
                "sesa_chunk_gather_constant_f32")
    return out


def ola_accumulate(y, starts, seg_lens, window, result, counter):
    """inference_pytorch.py:151-159 (in place on result/counter)."""
    y = _dev_f32(y, "sesa ola_accumulate")
    n_chunks, chunk = y.shape[0], y.shape[-1]
    n_out_ch = y[0].numel() // chunk
    if not (window.device == result.device == counter.device == y.device):
        raise N.SesaError("sesa ola_accumulate: y / window / result / counter must be on one device")
    with _on(y):
        N.check(N.lib().sesa_ola_accumulate_f32(y.data_ptr(), n_chunks, n_out_ch, chunk, N.i64_array(starts),
                                                N.i64_array(seg_lens), window.data_ptr(), result.data_ptr(),
                                                counter.data_ptr(), result.shape[-1], _stream(y)),
                "sesa_ola_accumulate_f32")


def ola_counter(chunk, starts, seg_lens, window, counter):
    """The counter half of inference_pytorch.py:158 only (n_out_ch = 0), in place."""
    counter = _dev_f32(counter, "sesa ola_counter")
    with _on(counter):
        N.check(N.lib().sesa_ola_accumulate_f32(None, len(starts), 0, chunk, N.i64_array(starts),
                                                N.i64_array(seg_lens), window.data_ptr(), None, counter.data_ptr(),
                                                counter.shape[-1], _stream(counter)), "sesa_ola_accumulate_f32")


def ola_finalize(result, counter, border):
    """inference_pytorch.py:174-180 -> [n_out_ch, L_pad - 2*border]."""
    n_out_ch, L_pad = result.shape
    out = torch.empty(n_out_ch, L_pad - 2 * border, device=result.device, dtype=torch.float32)
    with _on(result):
        N.check(N.lib().sesa_ola_finalize_f32(result.data_ptr(), counter.data_ptr(), n_out_ch, L_pad, border,
                                              out.data_ptr(), _stream(result)), "sesa_ola_finalize_f32")
    return out
