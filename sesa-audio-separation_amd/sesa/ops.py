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


# ---- chunker / overlap-add as custom ops (inference_pytorch.py:102-180) --------------------------------
# The functional forms return new tensors; the ``*_into`` / accumulate forms mutate their declared
# outputs (``mutates_args``), so torch.compile / functionalization see the real data flow.

@torch.library.custom_op("sesa::chunk_gather_into", mutates_args=("out",))
def _chunk_gather_into(mix: torch.Tensor, border: int, starts: list[int], chunk: int, out: torch.Tensor) -> None:
    mix = _dev_f32(mix, "sesa::chunk_gather")
    n_ch, L = mix.shape
    if out.shape != (len(starts), n_ch, chunk) or not out.is_contiguous() or out.device != mix.device:
        raise N.SesaError(f"sesa::chunk_gather: out must be contiguous [{len(starts)}, {n_ch}, {chunk}] on {mix.device}")
    with _on(mix):
        N.check(N.lib().sesa_chunk_gather_f32(mix.data_ptr(), n_ch, L, border, N.i64_array(starts), len(starts),
                                              chunk, out.data_ptr(), _stream(mix)), "sesa_chunk_gather_f32")


@_chunk_gather_into.register_fake
def _(mix, border, starts, chunk, out):
    return None


@torch.library.custom_op("sesa::chunk_gather", mutates_args=())
def _chunk_gather(mix: torch.Tensor, border: int, starts: list[int], chunk: int) -> torch.Tensor:
    out = torch.empty(len(starts), mix.shape[0], chunk, device=mix.device, dtype=torch.float32)
    _chunk_gather_into(mix, border, starts, chunk, out)
    return out


@_chunk_gather.register_fake
def _(mix, border, starts, chunk):
    return mix.new_empty(len(starts), mix.shape[0], chunk)


@torch.library.custom_op("sesa::chunk_gather_constant_into", mutates_args=("out",))
def _chunk_gather_constant_into(mix: torch.Tensor, starts: list[int], chunk: int, out: torch.Tensor) -> None:
    mix = _dev_f32(mix, "sesa::chunk_gather_constant")
    n_ch, L = mix.shape
    if out.shape != (len(starts), n_ch, chunk) or not out.is_contiguous() or out.device != mix.device:
        raise N.SesaError(f"sesa::chunk_gather_constant: out must be contiguous [{len(starts)}, {n_ch}, {chunk}]")
    with _on(mix):
        N.check(N.lib().sesa_chunk_gather_constant_f32(mix.data_ptr(), n_ch, L, N.i64_array(starts), len(starts),
                                                       chunk, out.data_ptr(), _stream(mix)),
                "sesa_chunk_gather_constant_f32")


@_chunk_gather_constant_into.register_fake
def _(mix, starts, chunk, out):
    return None


@torch.library.custom_op("sesa::ola_accumulate", mutates_args=("result", "counter"))
def _ola_accumulate(y: torch.Tensor, starts: list[int], seg_lens: list[int], window: torch.Tensor,
                    result: torch.Tensor, counter: torch.Tensor) -> None:
    y = _dev_f32(y, "sesa::ola_accumulate")
    n_chunks, chunk = y.shape[0], y.shape[-1]
    n_out_ch = y[0].numel() // chunk
    if not (window.device == result.device == counter.device == y.device):
        raise N.SesaError("sesa::ola_accumulate: y / window / result / counter must be on one device")
    with _on(y):
        N.check(N.lib().sesa_ola_accumulate_f32(y.data_ptr(), n_chunks, n_out_ch, chunk, N.i64_array(starts),
                                                N.i64_array(seg_lens), window.data_ptr(), result.data_ptr(),
                                                counter.data_ptr(), result.shape[-1], _stream(y)),
                "sesa_ola_accumulate_f32")


@_ola_accumulate.register_fake
def _(y, starts, seg_lens, window, result, counter):
    return None


@torch.library.custom_op("sesa::ola_counter", mutates_args=("counter",))
def _ola_counter(chunk: int, starts: list[int], seg_lens: list[int], window: torch.Tensor,
                 counter: torch.Tensor) -> None:
    counter = _dev_f32(counter, "sesa::ola_counter")
    with _on(counter):
        N.check(N.lib().sesa_ola_accumulate_f32(None, len(starts), 0, chunk, N.i64_array(starts),
                                                N.i64_array(seg_lens), window.data_ptr(), None, counter.data_ptr(),
                                                counter.shape[-1], _stream(counter)), "sesa_ola_accumulate_f32")


@_ola_counter.register_fake
def _(chunk, starts, seg_lens, window, counter):
    return None


@torch.library.custom_op("sesa::ola_finalize", mutates_args=())
def _ola_finalize(result: torch.Tensor, counter: torch.Tensor, border: int) -> torch.Tensor:
    result = _dev_f32(result, "sesa::ola_finalize")
    n_out_ch, L_pad = result.shape
    out = torch.empty(n_out_ch, L_pad - 2 * border, device=result.device, dtype=torch.float32)
    with _on(result):
        N.check(N.lib().sesa_ola_finalize_f32(result.data_ptr(), counter.data_ptr(), n_out_ch, L_pad, border,
                                              out.data_ptr(), _stream(result)), "sesa_ola_finalize_f32")
    return out


@_ola_finalize.register_fake
def _(result, counter, border):
    return result.new_empty(result.shape[0], result.shape[1] - 2 * border)


# ---- network forwards (one op per native network; the handle is the libsesa object pointer) ------------
def _network_forward(prefix, handle, x, workspace, out_shape):
    x = _dev_f32(x, f"sesa::{prefix}_forward")
    out = torch.empty(out_shape, device=x.device, dtype=torch.float32)
    with _on(x):
        N.check(getattr(N.lib(), f"sesa_{prefix}_forward")(handle, x.data_ptr(), x.shape[0], out.data_ptr(),
                                                            workspace.data_ptr(), workspace.numel(), _stream(x)),
                f"sesa_{prefix}_forward")
    return out


def _register_forward(prefix, ref):
    @torch.library.custom_op(f"sesa::{prefix}_forward", mutates_args=("workspace",))
    def fwd(handle: int, x: torch.Tensor, workspace: torch.Tensor, out_shape: list[int]) -> torch.Tensor:
        return _network_forward(prefix, handle, x, workspace, out_shape)

    fwd.__doc__ = f"Native {ref} forward on [B, ch, L] -> out_shape (libsesa sesa_{prefix}_forward)."

    @fwd.register_fake
    def _(handle, x, workspace, out_shape):
        return x.new_empty(out_shape)

    return fwd


mdx23c_forward = _register_forward("mdx23c", "MDX23C TFC_TDF_net (models/mdx23c_tfc_tdf_v3.py:161-242)")
bsr_forward = _register_forward("bsr", "BS-/Mel-Band-Roformer (models/bs_roformer.py:473-587)")
scnet_forward = _register_forward("scnet", "SCNet (models/scnet/scnet.py:316-374)")
htdemucs_forward = _register_forward("htdemucs", "HTDemucs (models/demucs4ht.py:548-693)")


# ---- Python entry points (same names / arguments as before; all go through the ops above) --------------
def chunk_gather(mix, border, starts, chunk, out=None):
    """inference_pytorch.py:102-103, :125-138 -> [n_chunks, n_ch, chunk]."""
    starts = [int(s) for s in starts]
    if out is None:
        return torch.ops.sesa.chunk_gather(mix, int(border), starts, int(chunk))
    torch.ops.sesa.chunk_gather_into(mix, int(border), starts, int(chunk), out)
    return out


def chunk_gather_constant(mix, starts, chunk, out=None):
    """utils.py:413-418 in demucs mode: no border pad, short chunks zero-padded -> [n_chunks, n_ch, chunk]."""
    starts = [int(s) for s in starts]
    if out is None:
        _dev_f32(mix, "sesa::chunk_gather_constant")
        out = torch.empty(len(starts), mix.shape[0], chunk, device=mix.device, dtype=torch.float32)
    torch.ops.sesa.chunk_gather_constant_into(mix, starts, int(chunk), out)
    return out


def ola_accumulate(y, starts, seg_lens, window, result, counter):
    """inference_pytorch.py:151-159 (in place on result/counter)."""
    torch.ops.sesa.ola_accumulate(y, [int(s) for s in starts], [int(s) for s in seg_lens], window, result, counter)


def ola_counter(chunk, starts, seg_lens, window, counter):
    """The counter half of inference_pytorch.py:158 only (n_out_ch = 0), in place."""
    torch.ops.sesa.ola_counter(int(chunk), [int(s) for s in starts], [int(s) for s in seg_lens], window, counter)


def ola_finalize(result, counter, border):
    """inference_pytorch.py:174-180 -> [n_out_ch, L_pad - 2*border]."""
    return torch.ops.sesa.ola_finalize(result, counter, int(border))
