"""Round 6: which kind of work is disturbed by a concurrent MFMA loop (tools/aggressors.hip)?  Each victim kernel (packed
f32 FMA chain, scalar FMA chain, LDS round trips) runs on the main stream over and over, its output compared bit for bit
with an idle-device run, while the side stream runs the given aggressor.

  python tools/victim_stress.py <victim: pk|fma|lds> <aggressor: none|mfma|...> [iters]
"""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dev = torch.device("cuda:0")


def main():
    vic, agg = sys.argv[1], sys.argv[2]
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    lib = ctypes.CDLL(os.path.join(REPO, "tools", "_canary", "libaggressors.so"))
    lib.agg_launch.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    lib.vic_launch.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_void_p]
    names = ["pk", "fma", "lds", "pkmix"] + [""] * 6 + ["st_pkmul", "st_pkadd", "st_pkfma", "st_scalar", "st_pkmul_nop",
                                                       "st_pkmul_global"] + [""] * 4 + [f"form{k}" for k in range(9)]
    vi = names.index(vic)
    blocks, vit = 512, {"pk": 4000, "fma": 4000, "lds": 200, "pkmix": 2000}.get(vic, 2000)
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    ref = torch.zeros(4 * blocks * 256, device=dev)
    lib.vic_launch(vi, blocks, vit, ctypes.c_void_p(ref.data_ptr()), ctypes.c_void_p(main_s.cuda_stream))
    torch.cuda.synchronize()
    fbuf = torch.zeros(1 << 22, device=dev)
    dbuf = torch.zeros(1 << 16, dtype=torch.float64, device=dev)
    outs, bad, nbad_elems = [], 0, []
    for it in range(iters):
        if agg != "none" and it % 2 == 0:
            ai = ["mfma", "atomic64", "atomic32", "lds", "epilogue"].index(agg)
            lib.agg_launch(ai, 1024, {"mfma": 20000}.get(agg, 500), ctypes.c_void_p(fbuf.data_ptr()),
                           ctypes.c_void_p(dbuf.data_ptr()), 1 << 16, ctypes.c_void_p(side.cuda_stream))
        o = torch.zeros_like(ref)
        lib.vic_launch(vi, blocks, vit, ctypes.c_void_p(o.data_ptr()), ctypes.c_void_p(main_s.cuda_stream))
        outs.append(o)
    torch.cuda.synchronize()
    for o in outs:
        ne = int((o.view(torch.int32) != ref.view(torch.int32)).sum())
        if ne:
            bad += 1
            nbad_elems.append(ne)
    if vic.startswith("st_"):   # these count their own mismatches: out[t] = number of stale stores seen by thread t
        tot = sum(int(o[:blocks * 256].view(torch.int32).sum()) for o in outs)
        print(f"   {vic}: {tot} stores carried a value other than the register result "
              f"(out of {iters * blocks * 256 * vit})", flush=True)
    print(f"RESULT victim={vic} aggressor={agg}: {bad} of {iters} outputs differ; differing elements per bad output "
          f"{sorted(nbad_elems)[:10]}", flush=True)


if __name__ == "__main__":
    main()
