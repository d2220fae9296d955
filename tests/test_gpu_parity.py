"""Parity of the HIP path (through the libsesa C ABI) against the reference's golden vectors and
the CPU oracle.  Needs a real MI355X: every test is marked ``gpu``.

Tolerances (written per test):
* integer/byte-like work (chunk gather, OLA accumulate/finalize given identical model output):
  bit-exact against the oracle restatement.
* STFT/iSTFT: fp32 FFT rounding, max |err| <= 2e-6 * max|X| (STFT) / 1e-6 abs (iSTFT).
* network / stems: per-sample RMS <= 1e-4 (north_star gate) in the default bf16x3 precision.
"""
import contextlib
import glob
import io
import os

import numpy as np
import pytest
import torch
import yaml

from conftest import CONFIGS, GOLDEN, rms

pytestmark = pytest.mark.gpu

RMS_GATE = 1e-4


def _cfg(name):
    from sesa.config import load_config
    return load_config("mdx23c", os.path.join(CONFIGS, name))


def _raw_cfg(name):
    with open(os.path.join(CONFIGS, name)) as f:
        return yaml.safe_load(f)


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda:0")


def _model(cfg_name, affine, precision="bf16x3", seed=0):
    from sesa.utils import get_model_from_config
    from sesa.weights import synth_state_dict
    m, c = get_model_from_config("mdx23c", os.path.join(CONFIGS, cfg_name))
    m.load_state_dict(synth_state_dict(m, affine=affine, seed=seed), strict=True)
    m.set_precision(precision)
    return m, c


def test_native_library_loaded():
    from sesa import _native
    assert _native.lib().sesa_version() >= 100


def test_stft_matches_reference(golden, dev):
    from sesa import ops
    g = golden("stft_istft.npz")
    x = torch.from_numpy(g["x"]).to(dev)                         # [1,2,16384]
    X = ops.stft(x, 8192, 1024, 4096)                             # [1,2,2,4096,17]
    X = X.reshape(1, 4, 4096, 17).cpu().numpy()
    ref = g["X"]
    assert np.abs(X - ref).max() <= 2e-6 * np.abs(ref).max()


def test_istft_matches_reference(golden, dev):
    from sesa import ops
    g = golden("stft_istft.npz")
    spec = torch.from_numpy(g["spec"]).to(dev).reshape(1, 2, 2, 2, 4096, 17)
    y = ops.istft(spec, 8192, 1024).reshape(g["y"].shape).cpu().numpy()
    assert np.abs(y - g["y"]).max() <= 1e-6


@pytest.mark.parametrize("L,border", [(40000, 0), (110250, 48384), (20000, 0)])
def test_chunk_gather_bit_exact(dev, L, border):
    from oracle import demix as od
    from sesa import ops
    rng = np.random.default_rng(5)
    mix = rng.standard_normal((2, L)).astype(np.float32)
    C, step = 64512, 16128
    L_pad = L + 2 * border
    mix_pad = np.pad(mix, ((0, 0), (border, border)), mode="reflect") if border else mix
    starts = list(range(0, L_pad, step))
    out = ops.chunk_gather(torch.from_numpy(mix).to(dev), border, starts, C).cpu().numpy()
    for j, s in enumerate(starts):
        np.testing.assert_array_equal(out[j], od.extract_chunk(mix_pad, s, C))


class _StandIn:
    """Deterministic stand-in model y = [x, -0.5x] (SURVEY §4 known-answer test)."""

    def __call__(self, x):
        return torch.stack([x, -0.5 * x], 1)


@pytest.mark.parametrize("L,bs", [(40000, 1), (40000, 2), (110250, 1), (110250, 3), (20000, 1), (300000, 2)])
def test_ola_bit_exact_vs_oracle(dev, L, bs):
    from oracle import demix as od
    from sesa.demix import demix_device
    c = _cfg("config_mdx23c_small.yaml")
    c.inference.batch_size = bs
    rng = np.random.default_rng(9)
    mix = (0.1 * rng.standard_normal((2, L))).astype(np.float32)
    with contextlib.redirect_stdout(io.StringIO()):
        est = demix_device(c, _StandIn(), mix, dev, exec_batch=3).cpu().numpy()
    ref = od.demix(c, lambda x: _StandIn()(x), mix, batch_size=bs)
    np.testing.assert_array_equal(est[0], ref["vocals"])
    np.testing.assert_array_equal(est[1], ref["other"])


@pytest.mark.parametrize("fixture,cfg_name", [("mdx23c_small.npz", "config_mdx23c_small.yaml"),
                                              ("mdx23c_small_vocals.npz", "config_mdx23c_small_vocals.yaml")])
def test_forward_small_matches_reference(golden, dev, fixture, cfg_name):
    g = golden(fixture)
    m, _ = _model(cfg_name, str(g["affine"]))
    y = m(torch.from_numpy(g["x"]).to(dev)).cpu().numpy()
    assert y.shape == g["y"].shape
    err = rms(y, g["y"])
    print(f"{fixture}: rms={err:.3e} ref_rms={rms(g['y'], 0 * g['y']):.3e}")
    assert err <= RMS_GATE


def test_forward_full_chunk_matches_reference(golden, dev):
    """The benchmark configuration (MDX23C vocals, 261120-sample chunk), bf16x3 precision."""
    g = golden("mdx23c_full_chunk.npz")
    m, _ = _model("config_vocals_mdx23c.yaml", "unit")
    y = m(torch.from_numpy(g["x"]).to(dev)).cpu().numpy()
    err = rms(y, g["y"])
    print(f"full chunk bf16x3: rms={err:.3e} max={np.abs(y - g['y']).max():.3e}")
    assert err <= RMS_GATE
    # batch invariance: the same chunk inside a batch of 3 gives the same output
    xb = torch.from_numpy(np.concatenate([g["x"], 0.5 * g["x"], g["x"]])).to(dev)
    yb = m(xb).cpu().numpy()
    assert rms(yb[0], y[0]) < 1e-7 and rms(yb[2], y[0]) < 1e-7


def test_forward_full_chunk_bf16_reports_deviation(golden, dev, record_property):
    """Throughput precision (--enable_amp / bench.py --precision bf16): measured and recorded, gated only
    loosely at 5e-3 (single-pass bf16 is expected near 6e-4, outside the 1e-4 parity gate -- the reference's
    own fp16 autocast is 1.35e-4).  The value is written to the junit report
    (record_property) and to gpurun_out/parity_bf16.json when that directory exists."""
    g = golden("mdx23c_full_chunk.npz")
    m, _ = _model("config_vocals_mdx23c.yaml", "unit", precision="bf16")
    y = m(torch.from_numpy(g["x"]).to(dev)).cpu().numpy()
    err = rms(y, g["y"])
    print(f"full chunk bf16: rms={err:.3e}")
    record_property("mdx23c_full_chunk_bf16_rms", err)
    out_dir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(out_dir):
        import json
        with open(os.path.join(out_dir, "parity_bf16.json"), "w") as f:
            json.dump({"fixture": "mdx23c_full_chunk.npz", "precision": "bf16", "rms_vs_reference": err,
                       "gate_bf16x3": RMS_GATE}, f)
    assert np.isfinite(y).all() and err < 5e-3


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "demix_small_*.npz"))),
                         ids=lambda p: os.path.basename(p))
def test_demix_matches_reference(dev, path):
    from sesa.backend import create_inference_session
    from sesa.demix import demix_pytorch_optimized
    g = np.load(path)
    m, c = _model("config_mdx23c_small.yaml", "random")
    c.inference.batch_size = int(g["batch_size"])
    be = create_inference_session(m, device="cuda:0", exec_batch=4)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        out = demix_pytorch_optimized(c, be, g["mix"], "cuda:0")
    prog = [ln for ln in buf.getvalue().splitlines() if ln.startswith("[SESA_PROGRESS]")]
    assert prog == list(g["progress"])
    for k in ("vocals", "other"):
        assert out[k].shape == g[k].shape
        assert rms(out[k], g[k]) <= RMS_GATE, k


@pytest.mark.parametrize("precision", ["bf16x3", "fp16mix"])
def test_side_streams_bit_identical(dev, precision):
    """streams > 1 (forwards overlapped on side streams, the OLA in chunk order on the main stream) is bit-identical
    to streams = 1, repeatedly.  Rounds 4-5 measured it differing (up to 1.6e-3): the FFT kernels' SLP-packed complex
    arithmetic -- v_pk_add_f32 / v_pk_mul_f32 with a source op_sel -- computed wrong columns while another stream's
    MFMA kernel shared their CUs (profiles/r06_pk_opsel_hazard.txt); libsesa is now built without those instructions
    (tools/isa_guard.py, tests/test_isa_guard.py).  Also: streams = 1 stays bit-identical run to run, and the
    workspace cache holds one entry per stream used."""
    from sesa.parallel import demix_sharded
    m, c = _model("config_mdx23c_small.yaml", "random", precision)
    rng = np.random.default_rng(2)
    mix = torch.from_numpy((0.1 * rng.standard_normal((2, 1200000))).astype(np.float32)).to(dev)
    a = demix_sharded(c, m, mix, dev, rank=0, world=1, exec_batch=3, streams=1)
    assert torch.equal(a, demix_sharded(c, m, mix, dev, rank=0, world=1, exec_batch=3, streams=1))
    assert len(m._ws) == 1
    for streams in (2, 3, 3, 2, 3):
        b = demix_sharded(c, m, mix, dev, rank=0, world=1, exec_batch=3, streams=streams)
        assert torch.equal(a, b), f"streams={streams}: max diff {float((a - b).abs().max()):.3e}"
    assert len(m._ws) == 3


def test_sharded_path_single_rank_matches_demix(dev):
    """bench.py's step (sesa/parallel.py at world 1) equals the plain device demix bit-for-bit."""
    from sesa.demix import demix_device
    from sesa.parallel import demix_sharded
    m, c = _model("config_mdx23c_small.yaml", "random")
    rng = np.random.default_rng(1)
    mix = torch.from_numpy((0.1 * rng.standard_normal((2, 300000))).astype(np.float32)).to(dev)
    with contextlib.redirect_stdout(io.StringIO()):
        a = demix_device(c, m, mix, dev, exec_batch=4)
    b = demix_sharded(c, m, mix, dev, rank=0, world=1, exec_batch=4)
    assert torch.equal(a, b)


@pytest.mark.parametrize("L", [0, 1, 7, 1000, 32256, 32257, 64512])
def test_demix_edge_lengths_vs_oracle(dev, L):
    """Empty, tiny and chunk-boundary lengths (reflect/zero tail pads, unpadded tracks), stand-in
    model: bit-exact against the oracle restatement of the reference loop."""
    from oracle import demix as od
    from sesa.demix import demix_device
    c = _cfg("config_mdx23c_small.yaml")
    rng = np.random.default_rng(L)
    mix = (0.1 * rng.standard_normal((2, L))).astype(np.float32)
    with contextlib.redirect_stdout(io.StringIO()):
        est = demix_device(c, _StandIn(), mix, dev, exec_batch=2).cpu().numpy()
    ref = od.demix(c, lambda x: _StandIn()(x), mix)
    assert est.shape == (2, 2, L)
    np.testing.assert_array_equal(est[0], ref["vocals"])
    np.testing.assert_array_equal(est[1], ref["other"])


@pytest.mark.parametrize("precision", ["bf16x3", "fp16", "fp16mix"])
def test_config0_demix_10s_full_model_matches_reference(dev, golden, precision):
    """BASELINE configs[0] end to end: the REAL reference demix_pytorch_optimized (full MDX23C vocals
    config, 10 s seed-0 mix, 13 chunks, batch_size 1; tests/golden/make_golden.py --only demix_full)
    against sesa.demix.demix_pytorch_optimized on the device: RMS <= 1e-4, identical progress lines --
    in the parity precision and in the fp16 TFC-conv precision the headline bench runs."""
    from sesa.backend import create_inference_session
    from sesa.demix import demix_pytorch_optimized
    g = golden("demix_full_10s.npz")
    m, c = _model("config_vocals_mdx23c.yaml", "unit", precision=precision)
    be = create_inference_session(m, device="cuda:0")
    m.set_precision(precision)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        out = demix_pytorch_optimized(c, be, g["mix"], "cuda:0")
    prog = [ln for ln in buf.getvalue().splitlines() if ln.startswith("[SESA_PROGRESS]")]
    assert prog == list(g["progress"])
    for k in ("vocals", "other"):
        err = rms(out[k], g[k])
        print(f"configs[0] 10 s {k} ({precision}): rms {err:.3e} (ref rms {rms(g[k], 0):.3e})")
        assert out[k].shape == g[k].shape == (2, 441000) and err <= RMS_GATE


@pytest.mark.parametrize("precision", ["bf16x3", "fp16", "fp16mix"])
def test_full_size_4min_properties(dev, precision):
    """configs[1] at full size (4-min track, full vocals config, 169 chunks): the sharded path at world 1
    equals demix_device bit-for-bit, the stems are finite and shaped [2, 2, L], and the two stems
    are not degenerate (size-independent properties; the oracle would need ~17 min of CPU)."""
    from sesa.demix import demix_device
    from sesa.parallel import demix_sharded
    m, c = _model("config_vocals_mdx23c.yaml", "unit", precision=precision)
    L = 240 * 44100
    rng = np.random.default_rng(0)
    mix = torch.from_numpy((0.1 * rng.standard_normal((2, L))).astype(np.float32)).to(dev)
    with contextlib.redirect_stdout(io.StringIO()):
        a = demix_device(c, m, mix, dev)
    b = demix_sharded(c, m, mix, dev, rank=0, world=1, exec_batch=57)
    assert a.shape == b.shape == (2, 2, L)
    assert torch.isfinite(a).all().item()
    assert torch.equal(a, b)
    assert float(a[0].std()) > 1e-4 and float((a[0] - a[1]).abs().max()) > 1e-4


def test_instancenorm_stress_large_offsets(dev, golden):
    """InstanceNorm with |mean| >> std (norm beta ~ U(2, 4), DC-offset input; reference golden
    tests/golden/mdx23c_small_stress.npz): the conv / TDF epilogues accumulate the statistics in
    fp64, so E[x^2] - E[x]^2 keeps its precision (mdx23c_tfc_tdf_v3.py:47-59)."""
    g = golden("mdx23c_small_stress.npz")
    m, _ = _model("config_mdx23c_small.yaml", "stress")
    y = m(torch.from_numpy(g["x"]).to(dev)).cpu().numpy()
    err = rms(y, g["y"])
    print(f"IN stress: rms {err:.3e} (ref rms {rms(g['y'], 0):.3e})")
    assert err <= RMS_GATE


@pytest.mark.parametrize("fixture,cfg_name,affine,mode", [
    ("mdx23c_small.npz", "config_mdx23c_small.yaml", None, 2),
    ("mdx23c_small_stress.npz", "config_mdx23c_small.yaml", "stress", 2),
    ("mdx23c_full_chunk.npz", "config_vocals_mdx23c.yaml", "unit", 1),
    ("mdx23c_full_chunk.npz", "config_vocals_mdx23c.yaml", "unit", 2)])
def test_conv3x3_wino_matches_reference(golden, dev, fixture, cfg_name, affine, mode):
    """The opt-in Winograd F(2, 3) TFC convs (conv3x3_wino_kernel; sesa_mdx23c_set_wino(mode), 1 = levels
    with 32 <= T <= 128, 2 = every T >= 32 level incl. the fused 1x1 shortcut stages) against the same
    reference goldens as the direct kernel.  The mode is read when the model is finalized, so the model
    is created under it."""
    from sesa import _native
    g = golden(fixture)
    prev = _native.lib().sesa_mdx23c_set_wino(mode)
    try:
        m, _ = _model(cfg_name, affine or str(g["affine"]))
        y = m(torch.from_numpy(g["x"]).to(dev)).cpu().numpy()
    finally:
        _native.lib().sesa_mdx23c_set_wino(prev)
    err = rms(y, g["y"])
    print(f"{fixture} (Winograd mode {mode}): rms={err:.3e}")
    assert err <= RMS_GATE
    m0, _ = _model(cfg_name, affine or str(g["affine"]))             # direct kernels, same weights
    y0 = m0(torch.from_numpy(g["x"]).to(dev)).cpu().numpy()
    assert rms(y0, y) <= 1e-5                                         # fp32 rounding / summation order only


@pytest.mark.parametrize("fixture,cfg_name,affine", [("mdx23c_small.npz", "config_mdx23c_small.yaml", None),
                                                     ("mdx23c_small_stress.npz", "config_mdx23c_small.yaml", "stress"),
                                                     ("mdx23c_full_chunk.npz", "config_vocals_mdx23c.yaml", "unit")])
def test_conv3x3_m16_variant_matches_reference(golden, dev, fixture, cfg_name, affine):
    """The opt-in conv3x3_m16_kernel (16x16x32 MFMA, persistent, LDS-DMA, shortcut from act_split raw
    planes; sesa_mdx23c_set_conv_variant(1)) against the same reference goldens as the default kernel."""
    from sesa import _native
    g = golden(fixture)
    m, _ = _model(cfg_name, affine or str(g["affine"]))
    prev = _native.lib().sesa_mdx23c_set_conv_variant(1)
    try:
        y = m(torch.from_numpy(g["x"]).to(dev)).cpu().numpy()
    finally:
        _native.lib().sesa_mdx23c_set_conv_variant(prev)
    err = rms(y, g["y"])
    print(f"{fixture} (m16 conv): rms={err:.3e}")
    assert err <= RMS_GATE
    y0 = m(torch.from_numpy(g["x"]).to(dev)).cpu().numpy()           # default kernel, same model
    assert rms(y0, y) <= 1e-5                                         # fp32 summation order only


@pytest.mark.parametrize("precision", ["fp16w2", "fp16", "fp16mix"])
@pytest.mark.parametrize("fixture,cfg_name,affine", [("mdx23c_small.npz", "config_mdx23c_small.yaml", None),
                                                     ("mdx23c_small_stress.npz", "config_mdx23c_small.yaml", "stress"),
                                                     ("mdx23c_full_chunk.npz", "config_vocals_mdx23c.yaml", "unit")])
def test_forward_fp16_conv_matches_reference(golden, dev, fixture, cfg_name, affine, precision, record_property):
    """SESA_PREC_F16W2 / SESA_PREC_F16: the direct TFC 3x3 convs (T >= 32 levels) on fp16 MFMA -- the
    activation rounded once to fp16 against fp16 hi + lo weights (fp16w2) or fp16 weights (fp16); every other
    contraction bf16x3.  Same 1e-4 per-sample RMS gate against the reference's fp32 goldens as the parity
    mode.  (CPU emulation of the same rounding on the full chunk, oracle/mdx23c.py with the 3x3 inputs
    rounded: 3.8e-5 for fp16w2, 5.2e-5 for fp16.)"""
    g = golden(fixture)
    m, _ = _model(cfg_name, affine or str(g["affine"]), precision=precision)
    y = m(torch.from_numpy(g["x"]).to(dev)).cpu().numpy()
    err = rms(y, g["y"])
    print(f"{fixture} ({precision} TFC convs): rms={err:.3e}")
    record_property(f"{fixture}_{precision}_rms", err)
    out_dir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(out_dir):
        import json
        with open(os.path.join(out_dir, f"parity_{precision}_{fixture.replace('.npz', '')}.json"), "w") as f:
            json.dump({"fixture": fixture, "precision": precision, "rms_vs_reference": err, "gate": RMS_GATE}, f)
    assert np.isfinite(y).all() and err <= RMS_GATE


# Full-width MDX23C goldens beyond the quiet white-noise chunk (tests/golden/make_golden.py --only full_levels):
# the SURVEY §8(d) seed-1 sines + noise signal, 0.3-RMS white noise (about -10 dBFS; the network's output and
# its rounding error both scale with the input level, mdx23c_tfc_tdf_v3.py:228-232), and a second weight draw.
FULL_FIXTURES = ["mdx23c_full_chunk.npz", "mdx23c_full_sines.npz", "mdx23c_full_loud.npz", "mdx23c_full_wseed2.npz"]


def _full_model(g, precision):
    seed = int(g["weight_seed"]) if "weight_seed" in g.files else 0
    return _model("config_vocals_mdx23c.yaml", str(g["affine"]), precision=precision, seed=seed)[0]


def _parity_stats(y, ref):
    d = np.asarray(y, np.float64) - ref
    err = float(np.sqrt(np.mean(d ** 2)))
    ref_rms = float(np.sqrt(np.mean(np.asarray(ref, np.float64) ** 2)))
    return {"rms": err, "rel_rms": err / ref_rms, "max_abs": float(np.abs(d).max()), "ref_rms": ref_rms}


# the precisions the product selects by default (bench headline / --enable_amp: fp16mix) and the parity and
# two-pass modes: every one gated at 1e-4 on every full-width fixture
@pytest.mark.parametrize("precision", ["bf16x3", "fp16w2", "fp16mix"])
@pytest.mark.parametrize("fixture", FULL_FIXTURES)
def test_full_chunk_levels_match_reference(golden, dev, fixture, precision):
    g = golden(fixture)
    m = _full_model(g, precision)
    y = m(torch.from_numpy(g["x"]).to(dev)).cpu().numpy()
    st = _parity_stats(y, g["y"])
    print(f"{fixture} {precision}: rms {st['rms']:.3e} rel {st['rel_rms']:.3e} max {st['max_abs']:.3e}")
    assert y.shape == g["y"].shape and np.isfinite(y).all() and st["rms"] <= RMS_GATE


def test_parity_matrix_report(golden, dev):
    """Every MDX23C precision on every full-width fixture: rms / rel_rms / max_abs written to
    gpurun_out/parity_matrix.json (evidence for DESIGN.md §4a); only finiteness is asserted here -- the
    gated modes are gated above, the single-pass fp16 / bf16 modes are reported (fp16 sits at the gate on the
    0.3-RMS fixture; CPU emulation 9.9e-5)."""
    import json
    out = {}
    for precision in ("bf16x3", "fp16w2", "fp16mix", "fp16", "bf16"):
        for fixture in FULL_FIXTURES:
            g = golden(fixture)
            m = _full_model(g, precision)
            y = m(torch.from_numpy(g["x"]).to(dev)).cpu().numpy()
            assert np.isfinite(y).all()
            out[f"{precision}/{fixture}"] = _parity_stats(y, g["y"])
            print(precision, fixture, out[f"{precision}/{fixture}"])
    out_dir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(out_dir):
        with open(os.path.join(out_dir, "parity_matrix.json"), "w") as f:
            json.dump(out, f, indent=1)
