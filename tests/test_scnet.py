"""SCNet on the native path.

CPU (no device work): the oracle restatement (oracle/scnet.py) against the golden vectors of the
real reference (tests/golden/make_golden_scnet.py); the Python and native parameter registries
both equal the reference state_dict keys; unsupported configurations are refused.  GPU (marked
``gpu``): the native forward / demix against the same golden vectors, per-sample RMS <= 1e-4
(north_star gate) in bf16x3 (the fp32 SIMT kernels are exact fp32; only the LSTM input / output
Linears run on MFMA); the bf16 throughput mode is measured and reported, not gated.
"""
import contextlib
import ctypes
import io
import json
import os

import numpy as np
import pytest
import torch

from conftest import CONFIGS, GOLDEN, rms

RMS_GATE = 1e-4


def _cfg(name):
    from oracle import scnet as osc
    return osc.load_cfg(os.path.join(CONFIGS, name))


def _model(cfg_name, affine="random", precision="bf16x3"):
    from oracle import scnet as osc
    from sesa.utils import get_model_from_config
    m, c = get_model_from_config("scnet", os.path.join(CONFIGS, cfg_name))
    sd = osc.synth_params(_cfg(cfg_name), affine)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    m.set_precision(precision)
    return m, c


@pytest.mark.parametrize("cfg_name,fx", [("config_scnet_small.yaml", "scnet_small.npz"),
                                         ("config_musdb18_scnet.yaml", "scnet_full_chunk.npz"),
                                         ("config_scnet_large_small.yaml", "scnet_large_small.npz"),
                                         ("config_scnet_wide_small.yaml", "scnet_wide_small.npz")])
def test_oracle_matches_reference(cfg_name, fx, golden):
    from oracle import scnet as osc
    g = golden(fx)
    cfg = _cfg(cfg_name)
    P = osc.to_torch(osc.synth_params(cfg, str(g["affine"])))
    with torch.inference_mode():
        y = osc.forward(P, cfg, torch.from_numpy(g["x"])).numpy()
    assert y.shape == g["y"].shape
    assert rms(y, g["y"]) <= 1e-6


@pytest.mark.parametrize("cfg_name,tag", [("config_musdb18_scnet.yaml", "musdb"), ("config_scnet_small.yaml", "small"),
                                          ("config_scnet_large_small.yaml", "large_small")])
def test_registry_matches_reference_state_dict(cfg_name, tag):
    from sesa import _native as N
    from sesa.utils import get_model_from_config
    m, c = get_model_from_config("scnet", os.path.join(CONFIGS, cfg_name))
    with open(os.path.join(GOLDEN, f"params_scnet_{tag}.json")) as f:
        ref = [(n, tuple(s)) for n, s in json.load(f)]
    assert [(n, tuple(t.shape)) for n, t in m.named_parameters()] == ref
    h = m._create(c.audio.chunk_size)          # host-side plan only: no device allocation
    try:
        names = []
        for i in range(N.lib().sesa_scnet_num_params(h)):
            nm, numel = ctypes.c_char_p(), ctypes.c_int64()
            assert N.lib().sesa_scnet_param_info(h, i, ctypes.byref(nm), ctypes.byref(numel)) == 0
            names.append((nm.value.decode(), numel.value))
    finally:
        N.lib().sesa_scnet_destroy(h)
    assert names == [(n, int(np.prod(s))) for n, s in ref]


def test_create_rejects_unsupported():
    from sesa import _native as N
    dims = (ctypes.c_int * 4)(4, 32, 64, 128)
    base = dict(chunk_size=485100, audio_channels=2, n_sources=4, n_fft=4096, hop_size=1024, win_size=4096,
                normalized=1, n_dims=4, dims=dims, band_sr=(ctypes.c_double * 3)(0.175, 0.392, 0.433),
                band_stride=(ctypes.c_int * 3)(1, 4, 16), band_kernel=(ctypes.c_int * 3)(3, 4, 16),
                conv_depths=(ctypes.c_int * 3)(3, 2, 1), compress=4, conv_kernel=3, num_dplayer=6, expand=1,
                precision=0)
    for bad, msg in ((dict(num_dplayer=5), b"num_dplayer"), (dict(n_fft=2048), b"nfft"),
                     (dict(conv_kernel=5), b"conv_kernel")):
        c = N.SesaScnetConfig(**{**base, **bad})
        h = ctypes.c_void_p()
        assert N.lib().sesa_scnet_create(ctypes.byref(c), ctypes.byref(h)) == -1
        assert msg in N.lib().sesa_last_error()
    c = N.SesaScnetConfig(**base)
    h = ctypes.c_void_p()
    assert N.lib().sesa_scnet_create(ctypes.byref(c), ctypes.byref(h)) == 0
    assert N.lib().sesa_scnet_workspace_size(h, 1) > 0
    N.lib().sesa_scnet_destroy(h)


def test_forward_refuses_cpu_tensor():
    from sesa import _native as N
    m, c = _model("config_scnet_small.yaml")
    with pytest.raises(N.SesaError):
        m(torch.zeros(1, 2, c.audio.chunk_size))


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda:0")


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16x3", "fp16mix"])
def test_forward_small_matches_reference(golden, dev, precision):
    g = golden("scnet_small.npz")
    m, _ = _model("config_scnet_small.yaml", str(g["affine"]), precision)
    y = m(torch.from_numpy(g["x"]).to(dev)).cpu().numpy()
    err = rms(y, g["y"])
    print(f"scnet small {precision} rms {err:.3e} (ref rms {rms(g['y'], 0):.3e})")
    assert y.shape == g["y"].shape and err <= RMS_GATE


# SCNet-large widths (registry "4STEMS-SCNet_Large", model.py:1347-1353; ConvolutionModule rows too wide
# for LDS, LSTM H = 512 on the odd dual-path layer) and an intermediate width (CM hidden 48, LSTM H 192 /
# 384): the wide kernels (scn_cm_*_gen_kernel, scn_lstm_mfma_wide_kernel) against the reference.
@pytest.mark.gpu
@pytest.mark.parametrize("cfg_name,fx", [("config_scnet_large_small.yaml", "scnet_large_small.npz"),
                                         ("config_scnet_wide_small.yaml", "scnet_wide_small.npz")])
def test_forward_wide_matches_reference(golden, dev, cfg_name, fx):
    g = golden(fx)
    m, _ = _model(cfg_name, str(g["affine"]))
    y = m(torch.from_numpy(g["x"]).to(dev)).cpu().numpy()
    err = rms(y, g["y"])
    print(f"{cfg_name} rms {err:.3e} (ref rms {rms(g['y'], 0):.3e})")
    assert y.shape == g["y"].shape and err <= RMS_GATE


@pytest.mark.gpu
def test_forward_small_bf16_reports_deviation(golden, dev):
    g = golden("scnet_small.npz")
    m, _ = _model("config_scnet_small.yaml", str(g["affine"]), precision="bf16")
    y = m(torch.from_numpy(g["x"]).to(dev)).cpu().numpy()
    err = rms(y, g["y"])
    print(f"scnet small bf16 rms {err:.3e} (reported, not gated)")
    assert np.isfinite(err) and err < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16x3", "fp16mix"])
def test_forward_full_chunk_matches_reference(golden, dev, precision):
    """fp16mix: the token GEMMs (3x3 convs, LSTM input projections, dual-path Linears) on one fp16 pass."""
    g = golden("scnet_full_chunk.npz")
    m, _ = _model("config_musdb18_scnet.yaml", str(g["affine"]), precision)
    y = m(torch.from_numpy(g["x"]).to(dev)).cpu().numpy()
    err = rms(y, g["y"])
    print(f"scnet musdb full chunk {precision} rms {err:.3e} (ref rms {rms(g['y'], 0):.3e})")
    assert err <= RMS_GATE


@pytest.mark.gpu
def test_forward_batch_items_independent(golden, dev):
    """Batch of 3 (two copies of item 0 around item 1): every item equals its own reference."""
    g = golden("scnet_small.npz")
    m, _ = _model("config_scnet_small.yaml", str(g["affine"]))
    x = np.stack([g["x"][0], g["x"][1], g["x"][0]])
    y = m(torch.from_numpy(x).to(dev)).cpu().numpy()
    for i, j in enumerate((0, 1, 0)):
        assert rms(y[i], g["y"][j]) <= RMS_GATE


@pytest.mark.gpu
def test_demix_matches_reference(golden, dev):
    from sesa.demix import demix_pytorch_optimized
    g = golden("demix_scnet_small.npz")
    m, c = _model("config_scnet_small.yaml", "random")
    with contextlib.redirect_stdout(io.StringIO()) as out:
        res = demix_pytorch_optimized(c, m, g["mix"], dev)
    prog = [ln for ln in out.getvalue().splitlines() if ln.startswith("[SESA_PROGRESS]")]
    assert prog == list(g["progress"])
    for k in c.training.instruments:
        assert res[k].shape == g[f"stem_{k}"].shape
        assert rms(res[k], g[f"stem_{k}"]) <= RMS_GATE


@pytest.mark.gpu
@pytest.mark.parametrize("L", [30001, 2049 * 3])
def test_forward_odd_lengths_match_oracle(dev, L):
    """Lengths that are not a multiple of the hop (scnet.py:330-333 right pad + crop), against the
    pinned oracle restatement on the same input."""
    from oracle import scnet as osc
    cfg = _cfg("config_scnet_small.yaml")
    m, _ = _model("config_scnet_small.yaml")
    P = osc.to_torch(osc.synth_params(cfg, "random"))
    x = (0.1 * np.random.default_rng(L).standard_normal((1, 2, L))).astype(np.float32)
    with torch.inference_mode():
        ref = osc.forward(P, cfg, torch.from_numpy(x)).numpy()
    y = m(torch.from_numpy(x).to(dev)).cpu().numpy()
    assert y.shape == ref.shape == (1, 4, 2, L)
    assert rms(y, ref) <= RMS_GATE


def test_feature_conversion_dft_matrices_match_numpy_fft():
    """scn_dft_mfma_kernel's formulation (sesa_scnet.hip finalize): FeatureConversion (separation.py:20-34, norm
    "ortho") as out = D @ in with rfft D = [s cos; -s sin] (2K x T, real parts then imaginary parts) and irfft
    D = [s w cos | -s w sin] (T x 2K, w = 1 at DC / Nyquist else 2, the imaginary DC / Nyquist columns zero).
    Checked here in float64 against numpy's FFTs -- the matrices the kernel packs (bf16 hi / lo) are these."""
    rng = np.random.default_rng(0)
    T, C = 18, 5
    K = T // 2 + 1
    s = 1.0 / np.sqrt(T)
    k = np.arange(K)[:, None]
    t = np.arange(T)[None, :]
    ang = 2 * np.pi * ((k * t) % T) / T
    Dr = np.concatenate([s * np.cos(ang), -s * np.sin(ang)], axis=0)          # [2K][T]
    x = rng.standard_normal((T, C))
    y = Dr @ x
    ref = np.fft.rfft(x, axis=0, norm="ortho")
    assert np.allclose(y[:K], ref.real, atol=1e-12) and np.allclose(y[K:], ref.imag, atol=1e-12)
    w = np.where((np.arange(K) == 0) | (np.arange(K) == K - 1), 1.0, 2.0)[None, :]
    edge = ((np.arange(K) == 0) | (np.arange(K) == K - 1))[None, :]
    angi = ang.T                                                                # [T][K]
    Di = np.concatenate([s * w * np.cos(angi), np.where(edge, 0.0, -s * w * np.sin(angi))], axis=1)   # [T][2K]
    spec_in = np.concatenate([ref.real, ref.imag], axis=0)                     # [2K][C]
    assert np.allclose(Di @ spec_in, x, atol=1e-12)
    # irfft ignores the imaginary parts of DC and Nyquist: so do the zero columns
    noisy = ref.copy()
    noisy[0] += 1j * rng.standard_normal(C)
    noisy[K - 1] += 1j * rng.standard_normal(C)
    noisy[1:K - 1] += rng.standard_normal((K - 2, C)) + 1j * rng.standard_normal((K - 2, C))
    back = Di @ np.concatenate([noisy.real, noisy.imag], axis=0)
    assert np.allclose(back, np.fft.irfft(noisy, n=T, axis=0, norm="ortho"), atol=1e-12)
