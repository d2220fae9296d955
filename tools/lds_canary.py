"""Round 6: catch LDS writes outside a workgroup's allocation.

tools/fft_stress.py showed the STFT kernel computing wrong (signal, frame) columns -- one workgroup's worth of bins --
while an MDX23C forward ran on another stream, and SESA_DEBUG_ONLY pinned the disturbing launches to the conv3x3 /
down / up / tdf classes.  This runs tools/lds_canary.hip's canary kernel (fills its LDS with a pattern, re-checks it)
on a side stream beside MDX23C forwards and prints what foreign writes it saw: LDS offsets and the values written,
which name the code that wrote them.

  python tools/lds_canary.py [model] [precision] [canary_lds_bytes] [iters]
"""
import ctypes
import os
import struct
import subprocess
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sesa-audio-separation_amd"), os.path.join(REPO, "tests"),
                os.path.join(REPO, "tools")]
LIB = os.path.join(REPO, "tools", "_canary", "liblds_canary.so")

dev = torch.device("cuda:0")


def load():
    if not os.path.exists(LIB):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                               os.path.join(REPO, "tools", "lds_canary.hip"), "-o", LIB])
    lib = ctypes.CDLL(LIB)
    lib.lds_canary_launch.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                           ctypes.c_void_p]
    return lib


def fmt(v):
    f = struct.unpack("<f", struct.pack("<I", v))[0]
    lo, hi = v & 0xFFFF, v >> 16
    bf = [struct.unpack("<f", struct.pack("<I", x << 16))[0] for x in (lo, hi)]
    return f"0x{v:08x} f32 {f:.4g} bf16 ({bf[0]:.4g}, {bf[1]:.4g})"


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "mdx23c"
    precision = sys.argv[2] if len(sys.argv) > 2 else "bf16x3"
    lds = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 30
    blocks = int(sys.argv[5]) if len(sys.argv) > 5 else 256      # ~one canary workgroup per CU: room beside it
    rounds = int(sys.argv[6]) if len(sys.argv) > 6 else 8000     # ~ the length of one small-config forward
    lib = load()
    from streams_trace import build
    m, c = build(kind, precision)
    rng = np.random.default_rng(3)
    xb = torch.from_numpy((0.1 * rng.standard_normal((3, 2, int(c.audio.chunk_size)))).astype(np.float32)).to(dev)
    m(xb)
    torch.cuda.synchronize()
    cap = 4096
    log = torch.zeros(4 * cap, dtype=torch.int32, device=dev)
    hits = torch.zeros(1, dtype=torch.int64, device=dev)
    side = torch.cuda.Stream(dev)
    for _ in range(iters):
        with torch.cuda.stream(side):
            lib.lds_canary_launch(blocks, lds, rounds, ctypes.c_void_p(log.data_ptr()), cap,
                                  ctypes.c_void_p(hits.data_ptr()), ctypes.c_void_p(side.cuda_stream))
        m(xb)
    torch.cuda.synchronize()
    n = int(hits.item())
    env = {k: v for k, v in os.environ.items() if k.startswith("SESA_")}
    print(f"RESULT lds_canary {kind} {precision} canary {lds} B env={env}: {n} foreign LDS writes seen", flush=True)
    if n:
        L = log.cpu().numpy().view(np.uint32).reshape(cap, 4)[:min(n, cap)]
        offs = L[:, 0]
        print(f"   offsets: min {offs.min()} max {offs.max()} distinct {len(set(offs.tolist()))}; "
              f"per-offset counts (first 16): {sorted(np.unique(offs, return_counts=True)[1].tolist())[-16:]}")
        uniq = {}
        for o, v, b, r in L:
            uniq.setdefault(int(o), []).append(int(v))
        for o in sorted(uniq)[:48]:
            vs = uniq[o]
            print(f"   +{o:6d}: {len(vs)} hits, e.g. {fmt(vs[0])}" + (f" | {fmt(vs[-1])}" if len(vs) > 1 else ""))


if __name__ == "__main__":
    main()
