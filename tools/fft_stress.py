"""Round 6: do the FFT kernels compute wrong values while another stream's forward runs beside them?

tools/streams_trace.py localised the multi-stream discrepancy to launches whose INPUT was bit-identical: the STFT and
the iSTFT (MDX23C and BS-Roformer, both precisions).  This stresses exactly that: stream A runs sesa::stft on one fixed
signal over and over (each output compared bit for bit with the idle-device result), while stream B runs network
forwards of the given model back to back.  Environment switches (SESA_TDF_VARIANT=old, SESA_TOKGEMM_GLDS=0, ...)
select which kernels stream B's forwards use.

  python tools/fft_stress.py [model|none] [precision] [iters]
"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sesa-audio-separation_amd"), os.path.join(REPO, "tests"),
                os.path.join(REPO, "tools")]
from sesa import ops  # noqa: E402

dev = torch.device("cuda:0")


def describe(o, ref):
    """Where a bad STFT output differs: o / ref [8, 2, 2 (re, im), 4096 bins, 256 frames]; one workgroup computes one
    (signal, frame) column."""
    d = (o - ref).abs().reshape(16, 2, 4096, -1)        # [signal, re/im, bin, frame]
    col = d.amax(dim=(1, 2)) > 0                          # [signal, frame]
    sig, fr = torch.nonzero(col, as_tuple=True)
    nbins = (d.amax(1) > 0).sum(1)                        # [signal, frame]: bins that differ
    pairs = list(zip(sig.tolist(), fr.tolist()))
    print(f"   bad output: {len(pairs)} (signal, frame) columns differ, e.g. {pairs[:6]}; bins differing per bad "
          f"column {sorted(set(int(nbins[s_, f_]) for s_, f_ in pairs))[:8]}; max |diff| {float(d.max()):.3e}",
          flush=True)


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "mdx23c"
    precision = sys.argv[2] if len(sys.argv) > 2 else "bf16x3"
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    rng = np.random.default_rng(5)
    x = torch.from_numpy((0.1 * rng.standard_normal((8, 2, 261120))).astype(np.float32)).to(dev)
    vlib = os.environ.get("FFT_VICTIM_LIB")   # another build of the spectral kernels as the victim (e.g. -fno-slp-vectorize)
    if vlib:
        import ctypes
        vl = ctypes.CDLL(os.path.join(REPO, vlib))
        vl.sesa_stft_f32.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 5 + [ctypes.c_void_p, ctypes.c_void_p]

        def stft(x_, n_fft, hop, dim_f):
            out = torch.empty(8, 2, 2, dim_f, 1 + x_.shape[-1] // hop, device=dev)
            assert vl.sesa_stft_f32(ctypes.c_void_p(x_.data_ptr()), 16, x_.shape[-1], n_fft, hop, dim_f,
                                    ctypes.c_void_p(out.data_ptr()),
                                    ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)) == 0
            return out
        ops.stft = stft
    ref = ops.stft(x, 8192, 1024, 4096).clone()
    torch.cuda.synchronize()
    side = torch.cuda.Stream(dev)
    m = xb = None
    big = torch.randn(4096, 4096, device=dev)
    if kind.startswith("agg:"):
        import ctypes
        lib = ctypes.CDLL(os.path.join(REPO, "tools", "_canary", "libaggressors.so"))
        lib.agg_launch.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        which = ["mfma", "atomic64", "atomic32", "lds", "epilogue"].index(kind[4:])
        fbuf = torch.zeros(1 << 22, device=dev)
        dbuf = torch.zeros(1 << 16, dtype=torch.float64, device=dev)
        iters_k = {"mfma": 20000, "atomic64": 2000, "atomic32": 2000, "lds": 200, "epilogue": 500}[kind[4:]]

        def side_work():
            lib.agg_launch(which, 1024, iters_k, ctypes.c_void_p(fbuf.data_ptr()), ctypes.c_void_p(dbuf.data_ptr()),
                           1 << 16, ctypes.c_void_p(side.cuda_stream))
    elif kind in ("matmul", "elementwise", "stft", "none"):
        def side_work():
            if kind == "matmul":
                return big @ big
            if kind == "elementwise":
                return (big * 1.0001 + 0.5).exp_()
            if kind == "stft":
                return ops.stft(x, 8192, 1024, 4096)
            return None
    else:
        from streams_trace import build
        m, c = build(kind, precision)
        C = int(c.audio.chunk_size)
        xb = torch.from_numpy((0.1 * rng.standard_normal((3, 2, C))).astype(np.float32)).to(dev)
        with torch.cuda.stream(side):
            m(xb)
        torch.cuda.synchronize()

        def side_work():
            return m(xb)
    bad, worst, t0 = 0, 0.0, time.time()
    outs = []
    for it in range(iters):
        if kind != "none" and it % 2 == 0:
            with torch.cuda.stream(side):
                side_work()      # keep the side stream busy
        y = ops.stft(x, 8192, 1024, 4096)
        outs.append(y)
        if len(outs) == 16:
            torch.cuda.synchronize()
            for o in outs:
                d = float((o - ref).abs().max())
                if d:
                    bad += 1
                    worst = max(worst, d)
                    if bad <= 3:
                        describe(o, ref)
            outs = []
    torch.cuda.synchronize()
    for o in outs:
        d = float((o - ref).abs().max())
        if d:
            bad += 1
            worst = max(worst, d)
    print(f"RESULT fft_stress side={kind} {precision} env="
          f"{ {k: v for k, v in os.environ.items() if k.startswith('SESA_')} }: {bad} of {iters} STFT outputs differ "
          f"(worst {worst:.3e}), {time.time() - t0:.1f} s", flush=True)


if __name__ == "__main__":
    main()
