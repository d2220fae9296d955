"""Round 6: localise the multi-stream discrepancy launch by launch.

Runs the chunk loop of sesa.parallel.local_accumulate_device (gather -> forward -> OLA, forwards alternating
between the main stream and side streams) on one track, with every MDX23C forward traced by libsesa's checksum hook
(sesa_debug_trace_begin / _end: a 64-bit checksum of each launch's output bytes, taken on the launch's own stream).
The streams = 1 run is the reference; each concurrent run reports, per forward group, the first launch whose
output checksum differs (and its kernel class) -- the launch that first produced a wrong value.

  python tools/streams_trace.py [model] [precision] [streams] [reps] [trace 0|1]
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sesa-audio-separation_amd"), os.path.join(REPO, "tests")]
from conftest import CONFIGS  # noqa: E402
from sesa import _native as N  # noqa: E402
from sesa import ops  # noqa: E402
from sesa.models import native as nat  # noqa: E402
from sesa.parallel import _runs, _Windows, shard_plan, side_streams  # noqa: E402
from sesa.utils import get_model_from_config  # noqa: E402
from sesa.weights import synth_model_state, synth_state_dict  # noqa: E402

dev = torch.device("cuda:0")
CAP = 8192
KCLS = ["conv3x3", "conv1x1", "down", "up", "tdf", "stft", "istft", "act", "tokgemm", "attn", "lstm", "simt", "ola",
        "hconv", "conv3x3_x3", "dft"]
CFG = {"mdx23c": "config_mdx23c_small.yaml", "bs_roformer": "config_bs_roformer_small.yaml",
       "scnet": "config_scnet_small.yaml", "htdemucs": "config_htdemucs_small.yaml"}


_orig_ws = nat.NativeModule.workspace


def zeroed_ws(self, device, h, batch):
    """The model's per-stream workspace, zeroed on the current stream before the forward: bytes a forward never
    writes then hold the same (zero) value in every run, so the per-launch workspace checksums compare only what the
    launches wrote."""
    ws = _orig_ws(self, device, h, batch)
    ws.zero_()
    return ws


def build(kind, precision):
    # STREAMS_TRACE_CONFIG=<yaml under tests/configs>: another config (the full-size ones) instead of CFG's small one
    m, c = get_model_from_config(kind, os.path.join(CONFIGS, os.environ.get("STREAMS_TRACE_CONFIG", CFG[kind])))
    m.load_state_dict(synth_state_dict(m, affine="random") if kind == "mdx23c" else
                      synth_model_state(m, affine="random"), strict=True)
    m.set_precision(precision)
    m.multi_stream_ok = True   # trace the raw behaviour
    return m, c


def run(m, c, mix, plan, rows, eb, streams, trace):
    lib = N.lib()
    C = plan["chunk"]
    n_ch = mix.shape[0]
    local = torch.zeros(rows, plan["span_max"], device=dev, dtype=torch.float32)
    scratch = torch.zeros(plan["span_max"], device=dev, dtype=torch.float32)
    lo, hi = plan["ranges"][0]
    s0 = plan["spans"][0][0]
    flat = plan["flat"]
    win = _Windows(plan, dev)
    main = torch.cuda.current_stream(dev)
    pool = [main] + side_streams(dev, streams - 1)
    xbufs, freed = [None] * len(pool), [None] * len(pool)
    traces = []
    for st in pool[1:]:
        st.wait_stream(main)
    pos, gi = lo, 0
    while pos < hi:
        grp = flat[pos:min(hi, pos + eb)]
        si = gi % len(pool)
        st = pool[si]
        if st is not main and freed[si] is not None:
            st.wait_event(freed[si])
        with torch.cuda.stream(st):
            if xbufs[si] is None or xbufs[si].shape[0] != len(grp):
                xbufs[si] = torch.empty(len(grp), n_ch, C, device=dev, dtype=torch.float32)
            xbuf = xbufs[si]
            if plan["mode"] == "demucs":
                ops.chunk_gather_constant(mix, [g[0] for g in grp], C, out=xbuf)
            else:
                ops.chunk_gather(mix, plan["border"], [g[0] for g in grp], C, out=xbuf)
            if trace:
                tb = torch.zeros(CAP, dtype=torch.int64, device=dev)
                N.check(lib.sesa_debug_trace_begin(ctypes.c_void_p(tb.data_ptr()), CAP), "trace_begin")
            y = m(xbuf).reshape(len(grp), rows, C)
            if trace:
                cls = (ctypes.c_int * CAP)()
                n = lib.sesa_debug_trace_end(cls, CAP)
                traces.append((tb, list(cls[:min(n, CAP)])))
        if st is not main:
            main.wait_stream(st)
            y.record_stream(main)
        for j, k in _runs(grp):
            ops.ola_accumulate(y[j:k], [g[0] - s0 for g in grp[j:k]], [g[1] for g in grp[j:k]],
                               win.pick(*grp[j][2:]), local, scratch)
        if st is not main:
            freed[si] = torch.cuda.Event()
            freed[si].record(main)
        pos += len(grp)
        gi += 1
    for st in pool[1:]:
        main.wait_stream(st)
    torch.cuda.synchronize()
    return local, [(t.cpu().numpy(), cl) for t, cl in traces]


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "mdx23c"
    precision = sys.argv[2] if len(sys.argv) > 2 else "bf16x3"
    streams = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    trace = bool(int(sys.argv[5])) if len(sys.argv) > 5 else kind == "mdx23c"
    if trace:
        nat.NativeModule.workspace = zeroed_ws
    m, c = build(kind, precision)
    mode = "demucs" if kind == "htdemucs" else "generic"
    rng = np.random.default_rng(2)
    L = int(sys.argv[6]) if len(sys.argv) > 6 else 1_200_000
    mix = torch.from_numpy((0.1 * rng.standard_normal((2, L))).astype(np.float32)).to(dev)
    plan = shard_plan(c, L, 1, mode)
    instr = list(c.training.instruments) if mode == "demucs" else (
        [c.training.target_instrument] if c.training.get("target_instrument") else list(c.training.instruments))
    rows = 2 * len(instr)
    eb = 3
    t0 = time.time()
    ref, rtr = run(m, c, mix, plan, rows, eb, 1, trace)
    ref2, rtr2 = run(m, c, mix, plan, rows, eb, 1, trace)
    print(f"[{kind} {precision}] {len(plan['flat'])} chunks, {len(rtr)} traced groups, "
          f"{len(rtr[0][1]) if rtr else 0} launches per forward; serial repeat max diff "
          f"{float((ref - ref2).abs().max()):.3e} ({time.time() - t0:.1f} s)", flush=True)
    if trace:
        for g, ((a, _), (b, _)) in enumerate(zip(rtr, rtr2)):
            if not np.array_equal(a, b):
                print(f"   serial repeat: group {g} trace differs at launches {np.nonzero(a != b)[0][:8].tolist()}")
    bad = 0
    firsts = {}
    for rep in range(reps):
        out, tr = run(m, c, mix, plan, rows, eb, streams, trace)
        d = float((out - ref).abs().max())
        if d == 0.0:
            continue
        bad += 1
        line = f"  rep {rep}: streams={streams} max diff {d:.3e}"
        if trace:
            for g, ((a, cl), (b, _)) in enumerate(zip(rtr, tr)):
                idx = np.nonzero(a != b)[0]
                if idx.size:
                    i0 = int(idx[0])
                    line += f"\n     group {g} (stream {g % streams}): first differing launch {i0} " \
                            f"({KCLS[cl[i0]] if i0 < len(cl) else '?'}), {idx.size} differ; next " \
                            f"{[(int(i), KCLS[cl[i]]) for i in idx[1:4]]}"
        print(line, flush=True)
        for g, ((a, cl), (b, _)) in enumerate(zip(rtr, tr)) if trace else []:
            idx = np.nonzero(a != b)[0]
            if idx.size:
                firsts[int(idx[0])] = firsts.get(int(idx[0]), 0) + 1
    print(f"RESULT {kind} {precision} streams={streams} trace={int(trace)}: {bad} of {reps} runs differ"
          + (f"; first-differing launch histogram {sorted(firsts.items())}" if firsts else "")
          + (f"; launch classes {[(i, KCLS[k]) for i, k in enumerate(rtr[0][1])]}" if trace and firsts else ""),
          flush=True)


if __name__ == "__main__":
    from sesa import parallel
    parallel._ALLOW_STREAMS = True
    main()
