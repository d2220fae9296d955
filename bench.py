#!/usr/bin/env python3
"""Benchmark: separated-audio seconds per wall second (x real-time) on MI355X (BASELINE.json metric;
default workload = configs[1]: MDX23C-TFC-TDF-v3 vocals, 4-min 44.1 kHz stereo track, chunked).

One "step" = one full pass of the hot path over the track: the mix resident in HBM -> chunk gather ->
native forward (exec_batch chunks per launch) -> device windowed overlap-add -> finalize -> stems in HBM
(the contract's `value`: inputs already resident when the timed region starts).  The same K steps are
timed again from the pinned host mix (H2D) to the stems in pinned host memory (D2H) and reported as
`pcie_inclusive` -- SURVEY §8(d)'s end-to-end wall time, never `value`.  With --gpus N (launched by
torch.distributed.run) the track's chunks are sharded contiguously over the N ranks and the spans are
gathered to rank 0 over RCCL (sesa/parallel.py); value = track seconds processed / max-over-ranks wall
time ("strong" scaling: one track, fixed total work).

Workloads (--model): mdx23c (configs[1], headline), bs_roformer (configs[2]), htdemucs (configs[3]:
30-min mix, utils.demix demucs-mode chunker, chunk-sharded), ensemble (configs[4]: mdx23c +
bs_roformer + scnet vocals blended on the device), scnet.

Also reported (rank 0):
* roofline -- the dominant kernel class, timed live in the timed region with hipEvents on the launch
  stream (libsesa sesa_profile_*): achieved = algorithmic FLOPs / kernel time; peak = dense bf16
  MFMA 2.5 PF/s divided by the MFMA passes per algorithmic FLOP (3 in bf16x3 parity precision);
  traffic = HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/pmc_<class>.json).
* cpu_baseline -- the CPU oracle (PyTorch-CPU fp32 restatement of the reference path, pinned to the
  reference's golden vectors) on a bounded sample of >= 8 chunks of the same workload, on every
  host core this process may use (N=1 only).
"""
import argparse
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "sesa-audio-separation_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

SR = 44100
CFG_DIR = os.path.join(REPO, "sesa-audio-separation_amd", "sesa", "configs")
# model -> (config, algorithmic FLOP per chunk, dominant kernel class or None (= most kernel time))
#   mdx23c: FlopCounterMode on the reference.
#   bs_roformer: FlopCounterMode on the reference for the Linears (addmm 5039 + mm 2500 GFLOP) plus
#          attention counted as 4 L^2 d per (sequence, head) -- QK^T + PV, the same definition the
#          attention class uses (FlopCounterMode saw only 104 GFLOP of it through SDPA): time
#          62 x 8 x 4 x 801^2 x 64 + freq 801 x 8 x 4 x 62^2 x 64, x 12 layers = 1053.3 GFLOP -> 8592.3 GFLOP.
#   scnet: FlopCounterMode on oracle/scnet.py (LSTM matmuls written out): conv 118.3 + LSTM input proj
#          128.4 + recurrence 128.4 + Linear 32.1 GFLOP per 485100-sample chunk.
#   htdemucs: FlopCounterMode on oracle/htdemucs.py (pinned to the reference class): conv 173.5 +
#          Linear 143.1 GFLOP, plus attention 4 Lq Lk d analytic (FlopCounterMode does not see the
#          CPU MHA fast path): 3 self layers (3792^2 + 1895^2) + 2 cross layers (2 x 3792 x 1895),
#          x 4 x 512 = 169.1 GFLOP -> 485.7 GFLOP per 485100-sample segment.
MODELS = {
    "mdx23c": ("config_vocals_mdx23c.yaml", 2.4341e12, "conv3x3"),
    "bs_roformer": ("config_bs_roformer_vocals.yaml", 8.5923e12, "tokgemm"),
    "scnet": ("config_musdb18_scnet.yaml", 4.072e11, None),
    "htdemucs": ("config_musdb18_htdemucs.yaml", 4.857e11, None),
}
ENSEMBLE = ("mdx23c", "bs_roformer", "scnet")
# forwards in flight per rank (sesa/parallel.py local_accumulate_device; re-entrant per stream since round 6).  Same box,
# --streams 1 vs 2 (profiles/r06_streams_ab.txt): HTDemucs 1282 -> 1342x (the 30-min track's 11 forwards overlap their
# low-occupancy tails), MDX23C 270.4 -> 274.2x, BS-Roformer 216.2 -> 219.8x (bit-identical to one stream since the
# iSTFT barrier fix); SCNet runs one forward per step.  The ensemble's members run one after another
# (--streams 2 gives each member two forwards in flight, ensemble_separate streams=; each member then plans its
# execution batch against the same free HBM, so it stays opt-in)
DEFAULT_STREAMS = {"htdemucs": 2, "mdx23c": 2, "bs_roformer": 2}
MODELS["ensemble"] = (None, sum(MODELS[m][1] for m in ENSEMBLE), None)
METRIC = {"ensemble": "separated-audio sec/sec (RTF), ensemble mdx23c + bs_roformer + scnet (vocals, avg_wave), MI355X",
          "mdx23c": "separated-audio sec/sec (RTF), MDX23C 44.1kHz stereo, 1/2/4/8 MI355X",
          "bs_roformer": "separated-audio sec/sec (RTF), BS-Roformer 44.1kHz stereo, MI355X",
          "scnet": "separated-audio sec/sec (RTF), SCNet 44.1kHz stereo, MI355X",
          "htdemucs": "separated-audio sec/sec (RTF), HTDemucs 44.1kHz stereo, 30-min mix chunk-sharded, MI355X"}
WORKLOAD = {"ensemble": "ensemble.py flow: mdx23c vocals + bs_roformer vocals + scnet musdb18, vocals stems "
                        "blended (sesa_blend_f32)",
            "mdx23c": "mdx23c_tfc_tdf_v3 vocals config",
            "bs_roformer": "bs_roformer (viperx 1297: dim 512, depth 12, 8x64 heads, 62 bands) vocals config",
            "scnet": "scnet musdb18 config (dims 4/32/64/128, 6 dual-path bi-LSTM layers, 4 sources)",
            "htdemucs": "demucs4ht htdemucs musdb18 config (channels 48, depth 4, bottom 512, 5 cross-transformer "
                        "layers, 4 sources)"}
HTD_MODE = {"generic": "live CLI chunker (inference.py -> demix_pytorch_optimized generic mode, chunk 485100, overlap 4)",
            "demucs": "utils.demix demucs mode (segment 11 s, overlap 4, no fades / border pad)"}
TRACK_SECONDS = {"htdemucs": 1800.0}
# chunks per forward: sesa.demix.plan_exec_batch (the CLI's planner): the model's cap, balanced so a
# rank's last forward is not a small remainder (169 chunks at N=1 -> 3 forwards of 57; 22 per rank at
# N=8 -> one forward of 22)
BF16_DENSE_TFLOPS = 2500.0  # MI355X_MICROARCH.md chip table (dense, no sparsity)
HBM_GBS = 8000.0            # MI355X_MICROARCH.md: HBM3E peak
FP32_VECTOR_TFLOPS = 157.3  # MI355X_MICROARCH.md chip table (fp32 vector)
KDESC = {"conv3x3": "conv3x3_db_kernel (TFC conv3x3, implicit GEMM, bf16x3 v_mfma_f32_32x32x16_bf16)",
         "tokgemm": "tok_gemm_glds_kernel + tok_gemm_kernel (token-major Linear layers, bf16x3 "
                    "v_mfma_f32_32x32x16_bf16 / v_mfma_f32_16x16x32_bf16)",
         "lstm": "scn_lstm_mfma_kernel / _wide_kernel (bi-LSTM recurrence: v_mfma_f32_32x32x16_f16, one fp16 pass in "
                 "SCNet fp16mix; bf16x3 v_mfma_f32_32x32x16_bf16 otherwise)",
         "dft": "scn_dft_mfma_kernel (SCNet feature conversion: rfft / irfft over T as a GEMM against the packed "
                "DFT matrix, bf16x3 v_mfma_f32_32x32x16_bf16)",
         "hconv": "tok_gemm_kernel<conv> (HTDemucs implicit-GEMM convolutions, v_mfma_f32_32x32x16_bf16)",
         "attn": "attn_kernel (flash attention, S^T = K Q^T, bf16x3 v_mfma_f32_32x32x16_bf16)",
         "simt": "norm / elementwise kernels priced at the fp32 VALU peak (SCNet: the ConvolutionModule layers -- "
                 "scn_cm_mfma_kernel in fp16mix, fp16 MFMA convs inside fp32 norms, else the VALU scn_cm_in / "
                 "scn_cm_out --, the dual-path GroupNorms, FeatureConversion fallbacks, the VALU band-conv fallback; "
                 "HTDemucs: htd_dc_conv_valu / htd_dc_gram / htd_dc_apply DConv, norms)"}


def kdesc(kclass, precision, model):
    """KDESC with the MFMA instruction of the precision the class's launches run in (class_precision)."""
    cp = class_precision(kclass, precision, model)
    if kclass == "conv3x3":
        cp = member_precision("mdx23c", precision, model)
        return {"bf16x3": KDESC["conv3x3"],
                "bf16": "conv3x3_db_kernel (TFC conv3x3, implicit GEMM, single-pass v_mfma_f32_32x32x16_bf16)",
                "fp16": "conv3x3_db_kernel<F16, MI4> (TFC conv3x3 T >= 32: one v_mfma_f32_32x32x16_f16 pass, "
                        "fused 1x1 shortcut bf16x3; T < 32: tap_gemm bf16x3)",
                "fp16w2": "conv3x3_db_kernel<F16 = 2> (TFC conv3x3 T >= 32: v_mfma_f32_32x32x16_f16 against fp16 "
                          "hi + lo weights, 2 passes; shortcut and T < 32 bf16x3)",
                "fp16mix": "conv3x3_db_kernel (TFC conv3x3 T >= 32 per level as the fp16mix plan: one "
                           "v_mfma_f32_32x32x16_f16 pass, or bf16x3 v_mfma_f32_32x32x16_bf16; shortcut and "
                           "T < 32 bf16x3)"}[cp]
    if kclass == "attn" and cp == "fp16":
        return ("attn_f16_kernel (flash attention, S^T = K Q^T, one v_mfma_f32_32x32x16_f16 pass for QK^T and PV, "
                "fp32 softmax statistics, double-buffered K / V)")
    if kclass == "hconv" and cp == "fp16":
        return ("tok_gemm_kernel<conv, F16> (HTDemucs implicit-GEMM convolutions and 1x1 rewrites, operand rounded "
                "once to fp16 in the staging, one v_mfma_f32_32x32x16_f16 pass)")
    if kclass == "tokgemm" and cp == "fp16":
        return ("tok_gemm_glds_kernel<EP_F16> (QKV / out-projection / FF Linears, one v_mfma_f32_16x16x32_f16 pass) + "
                "bf16x3 token GEMMs (band split, mask MLPs: v_mfma_f32_32x32x16_bf16 / 16x16x32_bf16)")
    if cp == "bf16" and kclass in KDESC:
        return KDESC[kclass].replace("bf16x3 ", "single-pass ")
    return KDESC[kclass]


# Sources that compile each kernel class: a committed PMC summary (profiles/pmc_<class>.json) counts only
# when it was measured on these exact sources (sha256 over their bytes; the GPU box has no .git).
_CSRC = os.path.join(REPO, "sesa-audio-separation_amd", "csrc")
_MDX_SRC = ("sesa_tapgemm.hip", "sesa_tapgemm.hpp", "sesa_common.hpp", "sesa_mdx23c.hip")
_TOK_SRC = ("sesa_tokgemm.hip", "sesa_tokgemm.hpp", "sesa_common.hpp")
KSRC = {"conv3x3": _MDX_SRC, "tdf": _MDX_SRC, "act": _MDX_SRC, "conv1x1": _MDX_SRC, "down": _MDX_SRC,
        "up": _MDX_SRC, "tokgemm": _TOK_SRC + ("sesa_bsroformer.hip",), "attn": _TOK_SRC + ("sesa_bsroformer.hip",),
        "hconv": _TOK_SRC + ("sesa_htdemucs.hip",), "lstm": ("sesa_scnet.hip", "sesa_tokgemm.hpp", "sesa_common.hpp"),
        "simt": ("sesa_scnet.hip", "sesa_common.hpp"), "dft": ("sesa_scnet.hip", "sesa_tokgemm.hpp", "sesa_common.hpp"),
        "conv3x3_x3": _MDX_SRC,
        "stft": ("sesa_spectral.hip", "sesa_common.hpp"), "istft": ("sesa_spectral.hip", "sesa_common.hpp"),
        "ola": ("sesa_ola.hip", "sesa_common.hpp")}


# each model's own source joins its classes' stamps (a class such as simt / tokgemm / attn has launches in several
# models, and their per-launch traffic differs): profiles/pmc_<class>_<model>.json
MODEL_SRC = {"mdx23c": ("sesa_mdx23c.hip",), "bs_roformer": ("sesa_bsroformer.hip",), "scnet": ("sesa_scnet.hip",),
             "htdemucs": ("sesa_htdemucs.hip",),
             "ensemble": ("sesa_mdx23c.hip", "sesa_bsroformer.hip", "sesa_scnet.hip")}


def kernel_sources_sha16(kclass, model=None):
    import hashlib
    h = hashlib.sha256()
    files = list(KSRC[kclass]) + ["Makefile"]   # (the build flags shape the code as much as the sources)
    for fn in MODEL_SRC.get(model, ()):
        if fn not in files:
            files.append(fn)
    for fn in files:
        with open(os.path.join(_CSRC, fn), "rb") as f:
            h.update(fn.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def default_precision(model):
    """MDX23C: fp16mix -- the T >= 32 TFC 3x3 convs on one fp16 MFMA pass except the encoder level-1 ones
    (bf16x3), the decoder TDF Linears fp16, the rest bf16x3: every MDX23C full-chunk golden (0.1-RMS noise,
    §8(d) sines, 0.3-RMS noise, a second weight draw) within 5.3e-5 of the reference; plain fp16 sits at
    9.75e-5 on the 0.3-RMS fixture, no margin.  BS-Roformer fp16: its QKV / out / FF Linears
    and attention on one fp16 pass.  HTDemucs fp16mix: attention, implicit-GEMM convs, 1x1 rewrites and the
    transformer / channel Linears on one fp16 pass (5.9e-6 full segment).  SCNet fp16mix: token GEMMs fp16,
    LSTM recurrence bf16x3 (9.7e-6 full chunk).  The ensemble's members run sesa.ensemble.ENSEMBLE_PRECISIONS
    (chosen so every configs[4] blend holds 8e-5).  Every line carries its measured parity."""
    return {"mdx23c": "fp16mix", "ensemble": "fp16mix", "bs_roformer": "fp16", "htdemucs": "fp16mix",
            "scnet": "fp16mix"}.get(model, "bf16x3")


# precision modes each native model accepts (sesa/models/*.py _precisions)
MODEL_PRECISIONS = {"mdx23c": ("bf16x3", "bf16", "fp16w2", "fp16", "fp16mix"), "bs_roformer": ("bf16x3", "bf16", "fp16"),
                    "scnet": ("bf16x3", "bf16", "fp16mix"), "htdemucs": ("bf16x3", "bf16", "fp16mix")}


def member_precision(name, precision, model=None):
    """The precision build_model gives member `name` of a `model` line run in `precision`: the ensemble's members
    their sesa.ensemble.ENSEMBLE_PRECISIONS for its default precision; otherwise fp16mix -> fp16 where the model
    has no fp16mix (BS-Roformer), and any mode the model lacks -> bf16x3 (e.g. fp16w2, MDX23C's only)."""
    if model == "ensemble" and precision == default_precision("ensemble"):
        from sesa.ensemble import ENSEMBLE_PRECISIONS
        return ENSEMBLE_PRECISIONS[name]
    if precision == "fp16mix" and precision not in MODEL_PRECISIONS[name]:
        precision = "fp16"
    return precision if precision in MODEL_PRECISIONS[name] else "bf16x3"


# kernel classes whose kernels run in the MDX23C precision mode
MDX_CLASSES = ("conv3x3", "conv3x3_x3", "conv1x1", "down", "up", "tdf", "act")


def class_precision(kclass, precision, model="mdx23c", members=None):
    """The arithmetic the launches of a kernel class run in, for a `model` line in `precision` (the roofline's MFMA
    pass count and the PMC stamp bench.py compares): ``members`` maps each member to the precision it actually built
    with (default: member_precision).  MDX23C classes follow MDX23C's mode; token GEMMs run one fp16 pass for a
    BS-Roformer fp16, SCNet fp16mix or HTDemucs fp16mix member (HTDemucs: unless SESA_HTD_PRESPLIT=0 keeps its
    Linears bf16x3), else that member's mode (bf16 / bf16x3); attention fp16 for BS-Roformer fp16 / HTDemucs
    fp16mix; HTDemucs' implicit-GEMM convs fp16 in fp16mix; the LSTM recurrence one fp16 pass in SCNet fp16mix
    (SESA_SCN_LSTM_PASSES), bf16 in the bf16 mode, else bf16x3;
    SCNet's feature-conversion DFTs bf16x3; simt is fp32 VALU."""
    if members is None:
        names = ("mdx23c", "bs_roformer", "scnet") if model == "ensemble" else (model,)
        members = {n: member_precision(n, precision, model) for n in names}
    if kclass in MDX_CLASSES:
        p = members.get("mdx23c", precision)
        if p not in ("fp16", "fp16w2", "fp16mix"):
            return p
        # the fp16 modes: conv3x3 = the one-pass (fp16w2: two-pass) fp16 direct convs; act = MDX23C's own mode
        # (its PMC stamp); fp16mix's TDF Linears mix fp16 (decoder) and bf16x3 stacks, priced at the fp16 peak (the
        # conservative choice); the fp16 up-convs (default since round 5; SESA_MDX_UP16=0 keeps them bf16x3); everything
        # else stays bf16x3
        if kclass == "conv3x3":
            return "fp16w2" if p == "fp16w2" else "fp16"
        if kclass == "act":
            return p
        if kclass == "tdf" and p == "fp16mix":
            return "fp16"
        if kclass == "up" and p == "fp16mix" and os.environ.get("SESA_MDX_UP16") != "0":
            return "fp16"
        return "bf16x3"
    if kclass == "simt":
        return "fp32"
    if kclass == "lstm":
        p = members.get("scnet")
        if p == "fp16mix":   # the fp16mix recurrence (H <= 256): SESA_SCN_LSTM_PASSES 1 (default) / 2 / 3
            return {"2": "fp16w2", "3": "bf16x3"}.get(os.environ.get("SESA_SCN_LSTM_PASSES", "1"), "fp16")
        return "bf16" if p == "bf16" else "bf16x3"
    if kclass == "dft":
        return "bf16x3"
    f16 = {"bs_roformer": "fp16", "scnet": "fp16mix", "htdemucs": "fp16mix"}
    users = {"tokgemm": ("bs_roformer", "scnet", "htdemucs"), "attn": ("bs_roformer", "htdemucs"),
             "hconv": ("htdemucs",)}.get(kclass, ())
    modes = set()
    for n in users:
        if n not in members:
            continue
        p = members[n]
        if p == f16[n] and not (n == "htdemucs" and kclass == "tokgemm" and os.environ.get("SESA_HTD_PRESPLIT") == "0"):
            modes.add("fp16")
        else:
            modes.add("bf16" if p == "bf16" else "bf16x3")
    # a class mixing one-pass fp16 and bf16x3 launches is priced at the one-pass peak (the conservative choice)
    return "fp16" if "fp16" in modes else (modes.pop() if len(modes) == 1 else "bf16x3")


def pmc_traffic(kclass, precision="bf16x3", model=None, records_per_step=None):
    """(HBM bytes per launch, provenance) from profiles/pmc_<class>_<model>.json when its ``src_sha16`` matches
    the kernel sources in this tree (the class's sources + the model's own) and it was measured in the same
    precision mode; (None, reason) otherwise -- a stale counter figure is not reported.
    A "launch" is one of libsesa's profile records -- the unit the algorithmic bytes are counted in.  Some records
    cover several kernel dispatches (SCNet's `simt` band convs: 9 per record; HTDemucs' DConv: 2), so with
    ``records_per_step`` (this run's records of the class per step) the counter bytes of one whole step are divided
    by it: traffic and algorithmic bytes then share one unit."""
    name = f"pmc_{kclass}_{model}.json" if model else f"pmc_{kclass}.json"
    pmc = os.path.join(REPO, "profiles", name)
    if not os.path.exists(pmc):
        return None, f"no profiles/{name}"
    with open(pmc) as f:
        d = json.load(f)
    cur = kernel_sources_sha16(kclass, model)
    if d.get("src_sha16") != cur:
        return None, (f"profiles/{name} measured on sources {d.get('src_sha16')} (git "
                      f"{d.get('git_sha', '?')}), this tree has {cur}: stale, not reported")
    if d.get("precision", "bf16x3") != precision:
        return None, (f"profiles/{name} measured in precision {d.get('precision', 'bf16x3')}, this run "
                      f"is {precision}: not reported")
    prov = {"file": f"profiles/{name}", "src_sha16": cur, "git_sha": d.get("git_sha"), "precision": precision,
            "algorithmic_bytes_per_launch": d.get("algorithmic_bytes_per_launch")}
    if records_per_step and d.get("hbm_bytes_per_step"):
        prov.update(counter_bytes_per_step=d["hbm_bytes_per_step"], dispatches_per_step=d.get("dispatches_per_step"),
                    records_per_step=round(records_per_step, 2),
                    unit="counter bytes of one step / libsesa records of the class per step")
        return round(d["hbm_bytes_per_step"] / records_per_step), prov
    return d.get("hbm_bytes_per_launch"), prov


def conv_plan_modes(precision, plan=None):
    """Per (side, level) mode of the direct (T >= 32) TFC 3x3 convs: '1' one fp16 pass, '2' fp16 x fp16 hi / lo
    weights, '3' bf16x3, 'b' single bf16 -- the SESA_PREC_F16MIX plan string of libsesa for fp16mix."""
    if precision == "fp16mix":
        return plan
    return {"fp16": "1", "fp16w2": "2", "bf16x3": "3", "bf16": "b"}[precision] * 16


def stream_counter_bytes(kclass, model, precision):
    """(HBM counter bytes per step, provenance) of a streaming class from profiles/pmc_<class>.json when it was
    measured on this tree's sources for the same workload (model, precision); (None, reason) otherwise."""
    pmc = os.path.join(REPO, "profiles", f"pmc_{kclass}.json")
    if not os.path.exists(pmc):
        return None, f"no profiles/pmc_{kclass}.json"
    with open(pmc) as f:
        d = json.load(f)
    if d.get("src_sha16") != kernel_sources_sha16(kclass):
        return None, f"profiles/pmc_{kclass}.json measured on other sources ({d.get('src_sha16')}): not reported"
    if (d.get("model"), d.get("precision")) != (model, precision):
        return None, f"profiles/pmc_{kclass}.json measured on {d.get('model')} / {d.get('precision')}: not reported"
    return d.get("hbm_bytes_per_step"), {"file": f"profiles/pmc_{kclass}.json", "git_sha": d.get("git_sha")}


def mdx23c_conv3x3_alg_bytes(cfg, batch, precision="bf16x3", plan=None):
    """Algorithmic HBM bytes of the conv3x3 class over one MDX23C forward of `batch` chunks, and its launch
    count (in the fp16 modes the class -- and so this count -- is the fp16 convs only; the bf16x3 ones are
    conv3x3_x3): each TFC 3x3 conv reads its input once -- fp32 for the fused-activation kernel (a bf16x3 / bf16
    conv with T >= 32, C_out <= 128), else the act_split planes: bf16 hi + lo 4 B, one fp16 (the fp16 modes)
    or bf16 plane 2 B -- the fused 1x1 shortcut's raw input (4 B) for conv2, and writes its fp32 output
    (4 B); weights per coefficient 4 B (bf16 hi + lo, fp16 hi + lo), 2 B (bf16 or fp16 alone); the T < 32
    convs run bf16x3 in every fp16 mode (mdx23c_tfc_tdf_v3.py:100-138; levels as TFC_TDF_net.__init__
    :141-203).  `plan`: the fp16mix plan (16 digits, encoder levels 0..7 then decoder levels 0..7)."""
    m = cfg.model
    n, nb, c0, g = int(m.num_scales), int(m.num_blocks_per_scale), int(m.num_channels), int(m.growth)
    T0, F0 = int(cfg.audio.dim_t), int(cfg.audio.dim_f) // int(m.num_subbands)
    modes = conv_plan_modes(precision, plan)
    f16mode = precision.startswith("fp16")   # then the conv3x3 class holds only the fp16 launches
    total, launches = 0.0, 0

    def stack(T, F, in_c, c, enc, lv):
        nonlocal total, launches
        pos = batch * T * F
        md = modes[(0 if enc else 8) + min(lv, 7)] if T >= 32 else ("b" if precision == "bf16" else "3")
        if f16mode and md not in "12":
            return
        if md in "12":
            a_in, wb = 2.0, (2.0 if md == "1" else 4.0)
        else:
            fused = T >= 32 and c <= 128
            a_in = 4.0 if (fused or md == "3") else 2.0
            wb = 2.0 if md == "b" else 4.0
        for i in range(nb):
            ic = in_c if i == 0 else c
            total += pos * ic * a_in + pos * c * 4.0 + 9 * ic * c * wb                     # conv1
            total += pos * c * a_in + pos * (c + ic) * 4.0 + 9 * c * c * wb + ic * c * 4.0  # conv2 (+ shortcut)
            launches += 2
    for lv in range(n):
        stack(T0 >> lv, F0 >> lv, c0 + g * lv, c0 + g * lv, True, lv)
    stack(T0 >> n, F0 >> n, c0 + g * n, c0 + g * n, True, n)
    for lv in reversed(range(n)):
        stack(T0 >> lv, F0 >> lv, 2 * (c0 + g * lv), c0 + g * lv, False, lv)
    return total, launches


def f16_plan():
    """libsesa's current SESA_PREC_F16MIX plan (16 digits; sesa_mdx23c_set_f16_plan query)."""
    import ctypes
    from sesa import _native
    buf = ctypes.create_string_buffer(17)
    _native.check(_native.lib().sesa_mdx23c_set_f16_plan(None, buf))
    return buf.value.decode()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cpu():
    """(threads this process may use, machine CPU count, CPU model string)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = min(avail, int(omp)) if omp and omp.isdigit() else avail
    model = platform.processor() or "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return threads, os.cpu_count(), model


def cpu_baseline(model_name, cfg_path, n_chunks_track, track_seconds, sample_chunks, config0=True):
    """Oracle (PyTorch-CPU fp32) forward on `sample_chunks` chunks of the workload; extrapolated to
    the track (OLA < 1 % of CPU time)."""
    threads, ncpu, cpu_model = host_cpu()
    torch.set_num_threads(threads)   # pytorch_backend.py:67-73 uses every core it has
    if model_name == "mdx23c":
        import yaml
        from oracle import mdx23c as om
        from oracle.weights import synth_state_dict
        with open(cfg_path) as f:
            cfg = yaml.safe_load(f)
        params = om.to_torch_params(synth_state_dict(om.param_shapes(cfg)))
        fwd = om.forward
        chunk = int(cfg["audio"]["chunk_size"])
    elif model_name == "scnet":
        from oracle import scnet as osc
        cfg = osc.load_cfg(cfg_path)
        params = osc.to_torch(osc.synth_params(cfg))
        fwd = osc.forward
        chunk = int(cfg["audio"]["chunk_size"])
    elif model_name == "htdemucs":
        import importlib.util
        from oracle import htdemucs as oh
        spec = importlib.util.spec_from_file_location("mgh", os.path.join(REPO, "tests", "golden",
                                                                          "make_golden_htdemucs.py"))
        mgh = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mgh)
        cfg = oh.load_cfg(cfg_path)
        params = oh.load(cfg, mgh.synth_params(dict(oh.param_names(cfg)), "random"))
        fwd = oh.forward
        chunk = int(cfg["training"]["samplerate"] * cfg["training"]["segment"])
    else:
        from oracle import bs_roformer as ob
        cfg = ob.load_cfg(cfg_path)
        params = ob.to_torch(ob.synth_params(cfg))
        fwd = ob.forward
        chunk = int(cfg["audio"]["chunk_size"])
    rng = np.random.default_rng(0)
    x = torch.from_numpy((0.1 * rng.standard_normal((1, 2, chunk))).astype(np.float32))
    if model_name == "mdx23c" and config0:
        # BASELINE.json configs[0] / BASELINE.md §4: the 10 s track timed END TO END on the CPU path --
        # chunker + forwards + windowed OLA (oracle/demix.py, inference_pytorch.py:55-186), batch_size 1
        # as the vocals config sets it; the per-chunk wall of that run then prices the 4-min workload
        from oracle.demix import demix as odemix
        mix10 = (0.1 * np.random.default_rng(0).standard_normal((2, int(10 * 44100)))).astype(np.float32)
        with torch.inference_mode():
            fwd(params, cfg, x)                   # warm-up (allocator, oneDNN primitives)
            t0 = time.time()
            n_seen = []
            odemix(cfg, lambda xb: fwd(params, cfg, xb), mix10, on_batch=lambda ch, y: n_seen.append(len(ch)))
            wall10 = time.time() - t0
        n10 = sum(n_seen)
        per_chunk = wall10 / n10
        return {"value": round(track_seconds / (per_chunk * n_chunks_track), 4), "unit": "separated-audio sec/sec",
                "cores": threads, "kind": "port",
                "host": {"cpu_model": cpu_model, "os_cpu_count": ncpu, "threads_used": threads},
                "config0_end_to_end": {"track_seconds": 10.0, "chunks": n10, "wall_s": round(wall10, 2),
                                       "value": round(10.0 / wall10, 4)},
                "sample": f"BASELINE configs[0]: 10 s 44.1 kHz stereo track (seed 0) separated end to end on the CPU "
                          f"path (oracle/demix.py chunker + OLA around oracle/mdx23c.py PyTorch-CPU fp32, full-width "
                          f"vocals config, {n10} chunks, {threads} threads) in {wall10:.1f} s = {10.0 / wall10:.4f}x "
                          f"real-time; value = that run's {per_chunk:.2f} s/chunk applied to the {n_chunks_track} "
                          f"chunks of the {track_seconds:.0f} s workload"}
    with torch.inference_mode():
        fwd(params, cfg, x)                       # warm-up (allocator, oneDNN primitives)
        t0 = time.time()
        for i in range(sample_chunks):
            fwd(params, cfg, x)
            # a progress line per chunk (stderr): a silent multi-minute CPU leg reads as a hung run
            print(f"[bench] cpu_baseline {model_name}: chunk {i + 1}/{sample_chunks} "
                  f"({time.time() - t0:.1f} s)", file=sys.stderr, flush=True)
    per_chunk = (time.time() - t0) / sample_chunks
    return {"value": round(track_seconds / (per_chunk * n_chunks_track), 4), "unit": "separated-audio sec/sec",
            "cores": threads, "kind": "port",
            "host": {"cpu_model": cpu_model, "os_cpu_count": ncpu, "threads_used": threads},
            "sample": f"{sample_chunks} of {n_chunks_track} chunks of the same {track_seconds:.0f} s track "
                      f"(after 1 warm-up chunk), full-width {model_name} config, oracle/{model_name}.py "
                      f"PyTorch-CPU fp32 on {threads} threads, {per_chunk:.2f} s/chunk, extrapolated per chunk "
                      f"(OLA <1% of CPU time, SURVEY §6)"}


# north_star parity, measured by the bench itself after the timed region: every benchmarked member, in the
# precision it ran, on the reference's own full-width outputs (tests/golden/make_golden*.py: the reference
# classes run in fp32 on CPU) -- MDX23C on four fixtures (0.1-RMS white noise, the SURVEY §8(d) seed-1 sines +
# noise signal, 0.3-RMS white noise, a second weight draw), the other models on their full-chunk golden
PARITY_FIXTURES = {"mdx23c": ["mdx23c_full_chunk.npz", "mdx23c_full_sines.npz", "mdx23c_full_loud.npz",
                              "mdx23c_full_wseed2.npz"],
                   "bs_roformer": ["bsr_full_chunk.npz"], "scnet": ["scnet_full_chunk.npz"],
                   "htdemucs": ["htdemucs_full_segment.npz"]}


def parity_leg(names, members, dev):
    from sesa.utils import get_model_from_config
    from sesa.weights import synth_model_state, synth_state_dict
    out, worst = {}, 0.0
    for nm, (model, _, cfg_path) in zip(names, members):
        for fx in PARITY_FIXTURES[nm]:
            g = np.load(os.path.join(REPO, "tests", "golden", fx), allow_pickle=False)
            affine = str(g["affine"]) if "affine" in g.files else "random"
            seed = int(g["weight_seed"]) if "weight_seed" in g.files else 0
            m, _ = get_model_from_config(nm, cfg_path)
            m.load_state_dict(synth_state_dict(m, affine=affine, seed=seed) if nm == "mdx23c" else
                              synth_model_state(m, affine=affine, seed=seed), strict=True)
            m.set_precision(model.precision)
            with torch.no_grad():
                y = m(torch.from_numpy(g["x"]).to(dev)).cpu().numpy().astype(np.float64)
            ref = g["y"].astype(np.float64)
            err = float(np.sqrt(np.mean((y - ref) ** 2)))
            ref_rms = float(np.sqrt(np.mean(ref ** 2)))
            out[fx] = {"model": nm, "precision": model.precision, "rms": err, "rel_rms": err / ref_rms,
                       "max_abs": float(np.abs(y - ref).max()), "ref_rms": ref_rms,
                       "input_rms": float(np.sqrt(np.mean(np.asarray(g["x"], np.float64) ** 2))),
                       "weight_seed": seed, "affine": affine}
            worst = max(worst, err)
            del m
    res = {"gate": 1e-4, "within_gate": worst <= 1e-4, "worst_rms": worst, "fixtures": out,
           "reference": "tests/golden/<fixture> (reference classes in fp32 on CPU, same name-keyed weights)"}
    if names == list(ENSEMBLE):
        res["blend"] = ensemble_blend_parity({nm: m.precision for nm, (m, _, _) in zip(names, members)}, dev)
        res["within_gate"] = res["within_gate"] and res["blend"]["worst_rms"] <= res["blend"]["gate"]
    return res


ENSEMBLE_FIXTURES = ("ensemble_full.npz", "ensemble_full_loud.npz", "ensemble_full_wseed2.npz")
BLEND_METHODS = ("avg_wave", "median_wave", "max_wave", "min_wave", "max_fft", "min_fft", "median_fft")


def ensemble_blend_parity(precisions, dev):
    """configs[4] blend parity: the three full-width members in the precisions the line ran, on the reference's own
    compositions (tests/golden/make_golden_ensemble_full.py: reference demix_pytorch_optimized per member, reference
    AudioEnsembleEngine blend) of a 0.1-RMS mix, the same mix at 0.3 RMS and a second weight draw -- every blend
    method (rms / rel / max), gated at 8e-5 (tests/test_ensemble_models.py)."""
    from sesa.ensemble import blend_device, ensemble_separate
    from sesa.utils import get_model_from_config
    from sesa.weights import synth_model_state, synth_state_dict
    out, worst = {}, 0.0
    for fx in ENSEMBLE_FIXTURES:
        g = np.load(os.path.join(REPO, "tests", "golden", fx), allow_pickle=False)
        seed = int(g["weight_seed"])
        members = []
        for nm in ENSEMBLE:
            m, c = get_model_from_config(nm, os.path.join(CFG_DIR, MODELS[nm][0]))
            aff = str(g[f"affine_{nm}"])
            m.load_state_dict(synth_state_dict(m, affine=aff, seed=seed) if nm == "mdx23c" else
                              synth_model_state(m, affine=aff, seed=seed), strict=True)
            m.set_precision(precisions[nm])
            members.append((c, m))
        blend0, stems = ensemble_separate(members, torch.from_numpy(g["mix"]).to(dev), "vocals", "avg_wave",
                                          weights=list(g["weights"]), rank=0, world=1, exec_batch=2)
        x = torch.stack([stems[i] for i in range(len(members))])
        rec = {"input_rms": float(np.sqrt(np.mean(np.asarray(g["mix"], np.float64) ** 2))), "weight_seed": seed}
        for i, nm in enumerate(ENSEMBLE):
            ref = g[f"vocals_{nm}"].astype(np.float64)
            y = stems[i].cpu().numpy().astype(np.float64)
            rec[f"stem_{nm}"] = {"rms": float(np.sqrt(np.mean((y - ref) ** 2)))}
        for meth in BLEND_METHODS:
            y = (blend0 if meth == "avg_wave" else blend_device(x, meth)).cpu().numpy().astype(np.float64)
            ref = g[f"blend_{meth}"].astype(np.float64)
            err = float(np.sqrt(np.mean((y - ref) ** 2)))
            rec[meth] = {"rms": err, "rel_rms": err / float(np.sqrt(np.mean(ref ** 2))),
                         "max_abs": float(np.abs(y - ref).max())}
            worst = max(worst, err)
        out[fx] = rec
        del members
    return {"gate": 8e-5, "worst_rms": worst, "precisions": precisions, "fixtures": out}


def synth_weights(model):
    """Name-keyed random-init weights with PyTorch's default-init bounds (no checkpoint offline)."""
    import zlib
    sd = {}
    shapes = dict(model.param_shapes())
    defaults = model.state_dict()
    for pname, shape in shapes.items():
        wname = pname[:-5] + ".weight" if pname.endswith(".bias") else pname.replace("bias_", "weight_")
        if len(shape) >= 2:
            fan_in = int(np.prod(shape[1:]))
        elif "bias" in pname and wname in shapes and len(shapes[wname]) >= 2:
            fan_in = int(np.prod(shapes[wname][1:]))
        else:                                                     # rotary freqs, norm gammas / betas, scales
            sd[pname] = defaults[pname]
            continue
        rng = np.random.Generator(np.random.PCG64(zlib.crc32(pname.encode()) ^ 0x5E5A))
        b = 1.0 / np.sqrt(fan_in)
        sd[pname] = torch.from_numpy(rng.uniform(-b, b, size=shape).astype(np.float32))
    return sd


def _forward_sizes(n_chunks, exec_batch, world):
    """Chunks per forward on rank 0: its contiguous share of the track, in exec_batch groups
    (sesa/parallel.py local_accumulate_device)."""
    per = -(-n_chunks // world)
    share = min(per, n_chunks)
    return [list(range(i, min(share, i + exec_batch))) for i in range(0, share, exec_batch)]


def build_model(name, precision, line_model=None):
    """Member `name` with name-keyed random-init weights, in member_precision(name, precision, line_model)."""
    from sesa.utils import get_model_from_config
    from sesa.weights import synth_state_dict
    cfg_path = os.path.join(CFG_DIR, MODELS[name][0])
    model, cfg = get_model_from_config(name, cfg_path)
    model.load_state_dict(synth_state_dict(model) if name == "mdx23c" else synth_weights(model), strict=True)
    model.set_precision(member_precision(name, precision, line_model))
    return model, cfg, cfg_path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--model", default="mdx23c", choices=sorted(MODELS))
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--precision", default=None, choices=["bf16x3", "bf16", "fp16w2", "fp16", "fp16mix"],
                    help="default: default_precision(model) -- fp16mix for mdx23c / ensemble, fp16 for bs_roformer, "
                         "else bf16x3")
    ap.add_argument("--exec-batch", type=int, default=0, help="chunks per forward (0: per-model default)")
    ap.add_argument("--track-seconds", type=float, default=0.0, help="0: 240 (1800 for htdemucs)")
    ap.add_argument("--cpu-sample-chunks", type=int, default=8)
    ap.add_argument("--blend", default="avg_wave", help="ensemble blend method (ensemble.py --type)")
    ap.add_argument("--htdemucs-mode", default="generic", choices=["generic", "demucs"],
                    help="htdemucs chunker: generic (the live CLI path, default) or utils.demix demucs mode")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the parity forward (PMC passes: one workload only)")
    ap.add_argument("--no-pcie", action="store_true",
                    help="skip the PCIe-inclusive timing (PMC / kernel-trace runs: the timed steps only)")
    ap.add_argument("--streams", type=int, default=None,
                    help="forwards in flight on separate HIP streams, bit-identical to 1 (sesa/parallel.py); default "
                         "per model (DEFAULT_STREAMS)")
    ap.add_argument("--rank-share", type=int, default=0, metavar="W",
                    help="one-GPU rehearsal of rank 0's share of a W-rank run (its chunks, its exec batch, local OLA + "
                         "finalise, no collective): value = the implied W-rank ceiling (track seconds / rank-0 time)")
    ap.add_argument("--gather", action="store_true",
                    help="multi-GPU: gather every rank's span to rank 0 (the round-5 form) instead of the owned form")
    ap.add_argument("--cpu-chunks-only", action="store_true",
                    help="mdx23c: time --cpu-sample-chunks forwards instead of the configs[0] 10 s end-to-end run")
    args = ap.parse_args()
    if args.precision is None:
        args.precision = default_precision(args.model)
    if args.streams is None:
        args.streams = DEFAULT_STREAMS.get(args.model, 1)
    track_seconds = args.track_seconds or TRACK_SECONDS.get(args.model, 240.0)

    from sesa.launch import needs_spawn, spawn_world, world_from_env
    if needs_spawn(args.gpus):
        # `python bench.py --gpus N` without torchrun: this parent has not touched HIP; it starts N
        # fresh rank processes under torch.distributed.run as a child and exits with its code
        log(f"bench: launching {args.gpus} ranks (torch.distributed.run, RCCL)")
        sys.exit(spawn_world(args.gpus, os.path.abspath(__file__), sys.argv[1:]))
    rank, local_rank, world = world_from_env()
    if world != args.gpus:
        log(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}; refusing to report a mismatched run")
        sys.exit(3)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        if dist.get_world_size() != args.gpus:
            log(f"bench: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
            sys.exit(3)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    from sesa import _native
    from sesa.demix import chunk_plan, demucs_chunk_plan
    from sesa.ensemble import ensemble_separate
    from sesa.parallel import demix_sharded

    names = list(ENSEMBLE) if args.model == "ensemble" else [args.model]
    members = [build_model(nm, args.precision, args.model) for nm in names]
    member_prec = {nm: m.precision for nm, (m, _, _) in zip(names, members)}
    n = int(round(track_seconds * SR))
    rng = np.random.default_rng(0)
    mix_host = torch.from_numpy((0.1 * rng.standard_normal((2, n))).astype(np.float32)).pin_memory()
    # htdemucs: "generic" = the live CLI path (inference.py -> demix_pytorch_optimized, generic chunker for
    # every model type, inference_pytorch.py:226); "demucs" = utils.demix(model_type='htdemucs')
    modes = [args.htdemucs_mode if nm == "htdemucs" else "generic" for nm in names]

    def n_chunks_of(cfg, mode):
        if mode == "demucs":
            return len(demucs_chunk_plan(n, int(cfg.training.samplerate * cfg.training.segment),
                                         int(cfg.inference.num_overlap)))
        return sum(len(b[0]) for b in chunk_plan(n, cfg.audio.chunk_size, cfg.inference.num_overlap,
                                                 cfg.inference.batch_size)[3])

    chunks = [n_chunks_of(cfg, md) for (_, cfg, _), md in zip(members, modes)]
    n_chunks = sum(chunks)

    from sesa.demix import plan_exec_batch

    def chunk_len(cfg, mode):
        return int(cfg.training.samplerate * cfg.training.segment) if mode == "demucs" else int(cfg.audio.chunk_size)

    sim = args.rank_share > 1 and world == 1      # rank 0's share of an args.rank_share-rank plan, on this GPU
    pworld = args.rank_share if sim else world    # the world size the chunk plan is sharded for
    batches = [args.exec_batch or plan_exec_batch(m, c, chunk_len(cfg, md), dev, world=pworld, streams=args.streams)
               for (m, cfg, _), c, md in zip(members, chunks, modes)]
    from sesa.parallel import shard_plan
    shard_ranges = [shard_plan(cfg, n, pworld, md)["ranges"] for (_, cfg, _), md in zip(members, modes)]
    path_flop = sum(c * MODELS[nm][1] for c, nm in zip(chunks, names))
    stems_host = None

    mix_dev = mix_host.to(dev)     # the track resident in HBM: `value`'s timed region starts from it
    # Multi-GPU (and its one-GPU rehearsal): the OWNED form (sesa/parallel.py demix_owned) -- each rank uploads only
    # the mix samples its chunks read, exchanges one seam with each neighbour and finalises its own output range,
    # which it copies to the host itself; no rank gathers the track.  The ensemble (members with different chunk
    # plans blended sample by sample) and plans with a rank shorter than one seam keep the gather to rank 0.
    from sesa.parallel import demix_owned, input_span, owned_ranges
    owned = (pworld > 1 and args.model != "ensemble" and not args.gather
             and owned_ranges(shard_plan(members[0][1], n, pworld, modes[0])) is not None)
    span = input_span(shard_plan(members[0][1], n, pworld, modes[0]), rank, n) if owned else (0, n)
    mix_span_buf = torch.empty_like(mix_dev) if owned else None

    def step(pcie=False):
        """One pass of the hot path over the track.  pcie=False (`value`): from the mix resident in HBM to the stems
        in HBM.  pcie=True (`pcie_inclusive`): pinned host mix -> H2D -> separation -> stems D2H (owned form: each
        rank moves only its input span and its own output range over its own PCIe link)."""
        nonlocal stems_host
        if pcie and owned:
            mix_span_buf[:, span[0]:span[1]].copy_(mix_host[:, span[0]:span[1]], non_blocking=True)
            mix_d = mix_span_buf
        else:
            mix_d = mix_host.to(dev, non_blocking=True) if pcie else mix_dev
        if args.model == "ensemble":
            est = ensemble_separate([(cfg, m) for m, cfg, _ in members], mix_d, "vocals", args.blend, rank=rank,
                                    world=pworld, exec_batch=batches, simulate=sim, streams=args.streams)[0]
        elif owned:
            m, cfg, _ = members[0]
            est = demix_owned(cfg, m, mix_d, dev, rank=rank, world=pworld, exec_batch=batches[0], mode=modes[0],
                              streams=args.streams, simulate=sim)[0]
        else:
            m, cfg, _ = members[0]
            est = demix_sharded(cfg, m, mix_d, dev, rank=rank, world=pworld, exec_batch=batches[0], mode=modes[0],
                                streams=args.streams, simulate=sim)
        if pcie and est is not None:   # stems D2H (gather form: rank 0's whole result; owned form: each rank's range)
            if stems_host is None or stems_host.shape != est.shape or stems_host.dtype != est.dtype:
                stems_host = torch.empty(est.shape, dtype=est.dtype, pin_memory=True)
            stems_host.copy_(est, non_blocking=True)
        return est

    for _ in range(args.warmup):
        step()
    if not args.no_pcie:
        step(pcie=True)            # (allocates the pinned stems buffer outside the timed regions)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # libsesa's per-launch event timing (the rooflines) runs inside the timed steps on one stream; with forwards in
    # flight on several streams an event pair would also time the other stream's kernels, so the rooflines then come
    # from a separate single-stream pass of the same K steps below (`roofline.timing_pass`)
    streams_timed = args.streams
    _native.profile_enable(streams_timed == 1)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        est = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    _native.profile_enable(False)
    if streams_timed > 1:
        args.streams = 1
        _native.profile_enable(True)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        _native.profile_enable(False)
        args.streams = streams_timed
    # the same K steps with the host transfers inside (reported as pcie_inclusive, never as `value`)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(0 if args.no_pcie else args.steps):
        step(pcie=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed_pcie = time.perf_counter() - t1
    if world > 1:
        t = torch.tensor([elapsed, elapsed_pcie], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, elapsed_pcie = (float(v) for v in t.tolist())
    assert owned or (est is None) == (rank != 0)
    if est is not None:
        assert torch.isfinite(est).all().item()
        assert args.no_pcie or (torch.isfinite(stems_host).all().item() and stems_host.shape == est.shape)

    # ---- rooflines of every kernel class, from libsesa's live hipEvent timing of the timed region ----
    # Each launch records its algorithmic FLOPs and algorithmic HBM bytes (operands read once, results written once,
    # in the storage types the launch reads / writes); a class's arithmetic intensity against the ridge of its own
    # compute peak picks its bound, and floor_frac = (sum over its launches of max(FLOP / peak, bytes / 8 TB/s)) /
    # its measured time -- the fraction of the roofline each launch's own intensity allows.
    passes_of = {"bf16x3": 3, "bf16": 1, "fp16w2": 2, "fp16": 1}

    def class_peak(kc):
        """(compute peak TFLOP/s, compute-bound name, note) of kernel class kc in this line's precisions."""
        cp = class_precision(kc, args.precision, args.model, member_prec)
        if cp == "fp32":
            return FP32_VECTOR_TFLOPS, "valu", "157.3 TF/s fp32 vector FMA peak (MI355X_MICROARCH.md; these kernels use no MFMA)"
        p = passes_of[cp]
        note = f"2.5 PF/s dense bf16/fp16 / {p} MFMA pass(es) per algorithmic FLOP ({cp})"
        if kc == "conv3x3" and member_prec.get("mdx23c") == "fp16mix":
            note += (f"; in fp16mix (plan {f16_plan()}) the conv3x3 class holds only the one-pass fp16 launches, the "
                     f"plan's bf16x3 levels are the conv3x3_x3 class")
        return BF16_DENSE_TFLOPS / p, "mfma", note

    def class_roof(kc):
        ms, n, work, nbytes = _native.profile_read2(kc)
        if not n or ms <= 0:
            return None
        peak_c, cbound, note = class_peak(kc)
        floor = _native.profile_floor(kc, peak_c, HBM_GBS)
        ridge = peak_c * 1e12 / (HBM_GBS * 1e9)                     # FLOP per byte
        ai = work / nbytes if nbytes > 0 else None
        hbm = ai is not None and ai < ridge
        r = {"bound": "hbm" if hbm else cbound,
             "achieved": round(nbytes / (ms * 1e-3) / 1e9, 1) if hbm else round(work / (ms * 1e-3) / 1e12, 2),
             "peak": HBM_GBS if hbm else round(peak_c, 1), "unit": "GB/s" if hbm else "TFLOP/s",
             "launches": n, "ms_per_step": round(ms / args.steps, 2), "avg_launch_ms": round(ms / n, 4),
             "flop_per_launch": round(work / n), "algorithmic_bytes_per_launch": round(nbytes / n) if nbytes else None,
             "flop_per_byte": round(ai, 1) if ai else None, "ridge_flop_per_byte": round(ridge, 1),
             "achieved_tflops": round(work / (ms * 1e-3) / 1e12, 2),
             "achieved_alg_gbs": round(nbytes / (ms * 1e-3) / 1e9, 1) if nbytes else None,
             "floor_ms_per_step": round(floor / args.steps, 2), "floor_frac": round(floor / ms, 4) if nbytes else None,
             "peak_note": note + (f"; HBM-side: {ai:.0f} FLOP/B < ridge {ridge:.0f}" if hbm else "")}
        r["frac"] = round(r["achieved"] / r["peak"], 4)
        return r

    compute_classes = ("conv3x3", "conv3x3_x3", "conv1x1", "down", "up", "tdf", "tokgemm", "attn", "lstm", "simt",
                       "hconv", "dft")
    roofs = {kc: rf for kc in compute_classes if (rf := class_roof(kc))}
    # dominant kernel class: the model's own, or the class with the most kernel time
    kclass = MODELS[args.model][2] or max(roofs, key=lambda k: roofs[k]["ms_per_step"])
    roof = dict(roofs[kclass])
    if pworld > 1:
        # the committed PMC summaries count one step of the N = 1 workload (its exec batch, its chunk count): a rank's
        # share has other launches and per-launch sizes, so its counter bytes are not known here
        traffic, traffic_src = None, (f"profiles/pmc_{kclass}_{args.model}.json counts the 1-GPU workload; not applied to "
                                      f"a {pworld}-rank share")
    else:
        traffic, traffic_src = pmc_traffic(kclass, class_precision(kclass, args.precision, args.model, member_prec),
                                           args.model, roof["launches"] / args.steps)
    if isinstance(traffic_src, dict):   # one algorithmic figure: this run's (the PMC file's own is for its run)
        traffic_src.pop("algorithmic_bytes_per_launch", None)
    alg_bytes = roof["algorithmic_bytes_per_launch"]
    if kclass == "conv3x3" and args.model == "mdx23c":
        # independent host-side model of the same bytes (mdx23c_conv3x3_alg_bytes) as a cross-check of libsesa's figure
        per_fwd, l_fwd = 0.0, 0
        for nb_ in [len(x) for x in _forward_sizes(chunks[0], batches[0], pworld)]:
            b_, l_ = mdx23c_conv3x3_alg_bytes(members[0][1], nb_, member_prec["mdx23c"], f16_plan())
            per_fwd += b_
            l_fwd += l_
        roof["algorithmic_bytes_host_model"] = round(per_fwd / max(l_fwd, 1))
    roof["timing_pass"] = ("the timed steps (one stream)" if args.streams == 1 else
                           f"a separate single-stream pass of the same {args.steps} steps (the timed steps ran "
                           f"{args.streams} streams)")
    roof.update(traffic=traffic, traffic_source=traffic_src, kernel=kdesc(kclass, args.precision, args.model),
                traffic_over_algorithmic=round(traffic / alg_bytes, 3) if traffic and alg_bytes else None,
                **{"class": kclass})
    path_tflops = path_flop * args.steps / elapsed / 1e12

    value = track_seconds * args.steps / elapsed
    if rank == 0:
        desc = []
        for nm, (_, cfg, _), c, eb, md in zip(names, members, chunks, batches, modes):
            C = int(cfg.training.samplerate * cfg.training.segment) if md == "demucs" else int(cfg.audio.chunk_size)
            mdesc = f", {HTD_MODE[md]}" if nm == "htdemucs" else ""
            desc.append(f"{WORKLOAD[nm]}{mdesc} (C={C}, overlap {int(cfg.inference.num_overlap)}, {c} chunks, "
                        f"exec batch {eb})")
        if args.model == "ensemble":
            desc = [WORKLOAD["ensemble"] + f" [{args.blend}]: " + "; ".join(desc)]
        line = {
            "metric": METRIC[args.model] + (f" -- rank-0 share of {pworld} ranks, one-GPU rehearsal" if sim else ""),
            "value": round(value, 3), "unit": "separated-audio sec/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None,
            "dtype": args.precision if len(names) == 1 else "+".join(f"{nm}:{member_prec[nm]}" for nm in names),
            # (rounds 1-4 and the first round-5 leases reported the PCIe-inclusive rate -- now `pcie_inclusive.value`
            # -- as `value`; from the last round-5 lease on, `value` is the HBM-resident rate, the bench contract's
            # "inputs already resident in HBM")
            "value_basis": "hbm_resident", "bench_contract_version": 2,
            "data": "synthetic: 0.1*N(0,1) stereo mix (seed 0), name-keyed random-init weights",
            "config": {"workload": f"{desc[0]}, {track_seconds:.0f} s 44.1 kHz stereo track chunked; timed: the mix "
                                   f"resident in HBM -> gather -> forwards -> OLA -> finalise -> stems in HBM "
                                   f"(pcie_inclusive adds the pinned host mix H2D and the stems D2H)",
                       "model": args.model, "chunks": n_chunks, "streams": args.streams,
                       "exec_batch": batches[0] if len(batches) == 1 else batches,
                       "parallelism": ((f"chunk-shard x{world}, owned ranges: per-rank input span H2D, RCCL seam "
                                        f"exchange with neighbours, per-rank finalise + D2H" if owned else
                                        f"chunk-shard x{world} + RCCL gather to rank 0") if world > 1 else
                                       f"1 GPU: rank 0's share of a {pworld}-rank chunk shard (rehearsal, no "
                                       f"collective; {'owned' if owned else 'gather'} form)" if sim else "1 GPU"),
                       "shard": {"world_size": dist.get_world_size() if world > 1 else 1,
                                 "backend": dist.get_backend() if world > 1 else None,
                                 "chunk_ranges": shard_ranges[0] if len(shard_ranges) == 1 else shard_ranges,
                                 **({"rehearsal_world": pworld} if sim else {})},
                       "path_tflops_algorithmic": round(path_tflops, 2)},
            "roofline": roof,
            "pcie_inclusive": None if args.no_pcie else {
                "value": round(track_seconds * args.steps / elapsed_pcie, 3),
                "ms_per_step": round(elapsed_pcie / args.steps * 1e3, 2),
                "note": ("same K steps from the pinned host mix (H2D) to the stems in pinned host memory (D2H), "
                         "transfers on the compute stream; " + ("owned form: each rank uploads its input span and "
                                                               "downloads its own output range" if owned else
                                                               "the whole mix to every rank, the stems from rank 0"))},
        }
        if sim:
            line["rehearsal"] = {
                "world": pworld, "rank0_chunks": shard_ranges[0][0][1] - shard_ranges[0][0][0] if len(names) == 1
                else [r[0][1] - r[0][0] for r in shard_ranges],
                "note": (f"value = track seconds / rank 0's wall time for its share (its input span -> forwards -> local "
                         f"OLA -> finalise of its own output range, no collective): the compute ceiling of a "
                         f"{pworld}-GPU run, which adds one RCCL seam exchange with each neighbour" if owned else
                         f"value = track seconds / rank 0's wall time for its share (gather -> forwards -> local OLA -> "
                         f"assemble + finalise, no collective): the compute ceiling of a {pworld}-GPU run, which "
                         f"adds the RCCL gather of the other ranks' spans to rank 0")}
        # north_star evidence: HBM GB/s of the streaming kernels (STFT / iSTFT / chunk gather + OLA),
        # algorithmic bytes / event-timed kernel time, against the 8 TB/s HBM3E peak
        hbm = {}
        for kc in ("stft", "istft", "ola", "act"):  # act: act_split (norm + GELU + bf16 hi/lo), 8 B/element
            kms, kn, kbytes = _native.profile_read(kc)
            if kn and kbytes > 0:
                gbs = kbytes / (kms * 1e-3) / 1e9
                hbm[kc] = {"achieved_gbs": round(gbs, 1), "frac": round(gbs / 8000.0, 4), "launches": kn,
                           "avg_launch_ms": round(kms / kn, 4), "bytes_per_launch": round(kbytes / kn)}
                # rocprofv3 counter bytes of one step of this workload (profiles/pmc_<class>.json, tools/pmc_stream.py);
                # act: the per-launch summary of tools/pmc_traffic.py (same sha / precision rules)
                if kc == "act":   # (measured on MDX23C's act_split / act_f16 launches: that model only)
                    bpl, src = (pmc_traffic("act", class_precision("act", args.precision, args.model), "mdx23c")
                                if args.model == "mdx23c" else (None, "act counters: measured for mdx23c only"))
                    cb = bpl * kn / args.steps if bpl else None
                else:
                    cb, src = stream_counter_bytes(kc, args.model, args.precision)
                hbm[kc]["counter_source"] = src
                if cb:
                    cgbs = cb * args.steps / (kms * 1e-3) / 1e9
                    hbm[kc].update(counter_bytes_per_step=cb, counter_gbs=round(cgbs, 1),
                                   counter_frac=round(cgbs / 8000.0, 4),
                                   counter_over_algorithmic=round(cb * args.steps / kbytes, 3))
        line["hbm_kernels"] = {"peak_gbs": 8000.0, **hbm}
        classes = {}
        for kc in ("conv3x3", "conv3x3_x3", "conv1x1", "down", "up", "tdf", "act", "tokgemm", "attn", "lstm", "simt",
                   "hconv", "dft", "stft", "istft", "ola"):
            kms, kn, kw = _native.profile_read(kc)
            if kn:
                classes[kc] = {"ms_per_step": round(kms / args.steps, 2), "launches": kn}
                if kc in roofs:   # the compute classes' own rooflines (bound by intensity, floor fraction)
                    classes[kc].update({k: roofs[kc][k] for k in ("bound", "achieved", "unit", "frac", "flop_per_byte",
                                                                   "floor_frac", "algorithmic_bytes_per_launch")})
                elif kc in hbm:
                    classes[kc].update(bound="hbm", achieved=hbm[kc]["achieved_gbs"], unit="GB/s", frac=hbm[kc]["frac"])
        line["kernel_classes"] = classes
        if "bs_roformer" in names or "htdemucs" in names:
            ams, alaunch, awork = _native.profile_read("attn")
            line["attention"] = {"kernel": kdesc("attn", args.precision, args.model),
                                 "achieved_tflops": round(awork / (ams * 1e-3) / 1e12, 2) if ams > 0 else 0.0,
                                 "launches": alaunch, "avg_launch_ms": round(ams / max(alaunch, 1), 4)}
        if not args.no_parity:
            line["parity"] = parity_leg(names, members, dev)
            line["parity_rms"] = line["parity"]["worst_rms"]
        if world == 1 and not args.no_cpu_baseline:
            parts = [cpu_baseline(nm, cp, c, track_seconds, args.cpu_sample_chunks,
                                  config0=len(names) == 1 and not args.cpu_chunks_only)
                     for nm, (_, _, cp), c in zip(names, members, chunks)]
            if len(parts) == 1:
                line["cpu_baseline"] = parts[0]
            else:  # the members run one after another: wall times add
                line["cpu_baseline"] = {
                    "value": round(track_seconds / sum(track_seconds / p["value"] for p in parts), 4),
                    "unit": "separated-audio sec/sec", "cores": parts[0]["cores"], "kind": "port",
                    "host": parts[0]["host"],
                    "sample": " + ".join(p["sample"] for p in parts) + "; member wall times summed"}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
