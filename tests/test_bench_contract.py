"""bench.py host logic (no GPU): the precision each model's default line runs in, and the conv3x3
algorithmic-bytes model that roofline.traffic is compared against."""
import os
import sys
from types import SimpleNamespace as NS

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def _vocals_cfg():
    # config_vocals_mdx23c.yaml: dim_f 4096 / 4 subbands, dim_t 256, 4 scales, 128 + 128 per level
    return NS(model=NS(num_scales=4, num_blocks_per_scale=1, num_channels=128, growth=128, num_subbands=4),
              audio=NS(dim_t=256, dim_f=4096))


def test_default_precision():
    assert bench.default_precision("mdx23c") == bench.default_precision("ensemble") == "fp16mix"
    assert bench.default_precision("bs_roformer") == "fp16"
    for m in ("htdemucs", "scnet"):
        assert bench.default_precision(m) == "fp16mix"
    # PMC stamps / roofline pass counts: the arithmetic each class's launches run in
    cp = bench.class_precision
    assert cp("hconv", "fp16mix", "htdemucs") == "fp16"
    assert cp("attn", "fp16mix", "htdemucs") == "fp16"
    assert cp("tokgemm", "fp16mix", "htdemucs") == "fp16"       # HTDemucs fp16mix Linears: one fp16 pass
    assert cp("tokgemm", "fp16mix", "scnet") == "fp16"
    assert cp("lstm", "fp16mix", "scnet") == "fp16"               # one fp16 recurrence pass (SESA_SCN_LSTM_PASSES=1)
    assert cp("lstm", "bf16x3", "scnet") == "bf16x3" and cp("lstm", "bf16", "scnet") == "bf16"
    assert cp("simt", "fp16mix", "scnet") == "fp32"              # VALU kernels
    assert cp("dft", "fp16mix", "scnet") == "bf16x3"             # feature-conversion DFTs on MFMA
    assert cp("conv3x3", "fp16") == "fp16" and cp("conv3x3", "fp16mix") == "fp16"
    assert cp("conv3x3", "fp16w2") == "fp16w2" and cp("conv3x3_x3", "fp16mix") == "bf16x3"
    assert cp("tdf", "fp16mix") == "fp16" and cp("tdf", "fp16") == "bf16x3" and cp("act", "fp16mix") == "fp16mix"
    assert cp("tokgemm", "fp16", "bs_roformer") == "fp16"
    assert cp("tokgemm", "fp16w2", "bs_roformer") == "bf16x3"     # BS-Roformer has no fp16w2: built bf16x3
    assert cp("attn", "fp16mix", "ensemble") == "fp16"
    assert cp("attn", "fp16", "htdemucs") == "bf16x3"
    assert cp("hconv", "fp16", "ensemble") == "bf16x3"
    assert cp("tokgemm", "bf16", "bs_roformer") == "bf16"
    assert cp("conv3x3", "bf16x3") == "bf16x3"
    # the members a line actually built decide (bench.py passes them)
    assert cp("tokgemm", "fp16mix", "ensemble", {"mdx23c": "bf16x3", "bs_roformer": "bf16x3", "scnet": "bf16x3"}) == "bf16x3"
    assert cp("conv3x3", "fp16mix", "ensemble", {"mdx23c": "bf16x3", "bs_roformer": "fp16", "scnet": "fp16mix"}) == "bf16x3"


def test_member_precision():
    from sesa.ensemble import ENSEMBLE_PRECISIONS
    for m in ("mdx23c", "bs_roformer", "scnet"):
        assert bench.member_precision(m, "fp16mix", "ensemble") == ENSEMBLE_PRECISIONS[m]
    assert bench.member_precision("bs_roformer", "fp16mix") == "fp16"
    assert bench.member_precision("scnet", "fp16") == "bf16x3"
    assert bench.member_precision("mdx23c", "fp16w2") == "fp16w2"
    assert bench.member_precision("htdemucs", "fp16w2") == "bf16x3"


def test_conv3x3_alg_bytes_by_precision():
    c = _vocals_cfg()
    b3, n3 = bench.mdx23c_conv3x3_alg_bytes(c, 57, "bf16x3")
    bw, nw = bench.mdx23c_conv3x3_alg_bytes(c, 57, "fp16w2")
    b1, n1 = bench.mdx23c_conv3x3_alg_bytes(c, 57, "fp16")
    assert n3 == 2 * 9                                    # 9 TFC_TDF stacks x (conv1, conv2)
    assert nw == n1 == 2 * 8                              # fp16 modes: the class is the T >= 32 fp16 convs only
    assert b1 / n1 < bw / nw                              # 2 B weights instead of 4
    # fp16mix: the plan's '3' levels leave the class (they are conv3x3_x3)
    bm, nm = bench.mdx23c_conv3x3_alg_bytes(c, 57, "fp16mix", "1311111111111111")
    assert nm == 2 * 7 and bm < b1                       # encoder level 1 (one block here) leaves
    # level 0 (fused fp32 input) is precision-independent apart from the weights
    b3_l0 = 57 * 256 * 1024 * (128 * 4 + 128 * 4) + 9 * 128 * 128 * 4
    assert b3 > 2 * b3_l0


def test_fp16_modes_are_mdx23c_only():
    from sesa.models.mdx23c import TFC_TDF_net
    from sesa.models.native import NativeModule
    assert "fp16" in TFC_TDF_net._precisions and "fp16mix" in TFC_TDF_net._precisions
    assert TFC_TDF_net._amp_precision == "fp16mix"
    assert "fp16" not in NativeModule._precisions and NativeModule._amp_precision == "bf16"


@pytest.mark.parametrize("name", ["bs_roformer", "scnet", "htdemucs"])
def test_bench_maps_fp16_to_parity_for_other_members(name, monkeypatch):
    seen = {}

    class Fake:
        def load_state_dict(self, *a, **k):
            pass

        def set_precision(self, p):
            seen["p"] = p

    import sesa.utils
    monkeypatch.setattr(sesa.utils, "get_model_from_config", lambda n, p: (Fake(), None))
    monkeypatch.setattr(bench, "synth_weights", lambda m: {})
    bench.build_model(name, "fp16w2")
    assert seen["p"] == "bf16x3"


def test_scnet_lstm_pass_switch(monkeypatch):
    """SESA_SCN_LSTM_PASSES selects the fp16mix recurrence's MFMA passes (sesa_scnet.hip scn_lstm_passes); the line
    prices the lstm class at the matching peak."""
    cp = bench.class_precision
    for env, want in (("1", "fp16"), ("2", "fp16w2"), ("3", "bf16x3")):
        monkeypatch.setenv("SESA_SCN_LSTM_PASSES", env)
        assert cp("lstm", "fp16mix", "scnet") == want
    monkeypatch.setenv("SESA_SCN_LSTM_PASSES", "3")
    assert cp("lstm", "bf16", "scnet") == "bf16"
