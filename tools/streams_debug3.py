"""Diagnostic 3 (round 5): why did local_accumulate_device(streams=2) differ from streams=1?

profiles/r04_streams_debug.txt: streams=2 changed samples 36800-43999 (group 0's span, chunks 0-2, main
stream) by up to 9.3e-4.  This script re-runs the same loop with hooks and records, per group:
  * the gathered input x (cloned on its stream right after the gather),
  * the forward output y (cloned on its stream right after the forward),
and then reports, for several schedules, which groups' x / y / final local buffers differ from the
single-stream run:
  A  streams=1                                   (reference)
  B  streams=2                                   (as in round 4)
  C  streams=2, host sync after every group      (no concurrency; same allocation pattern as B)
  D  streams=2, NaN guard bands around the workspaces and input buffers
  E  streams=2, y cloned into a fresh main-stream buffer before the OLA
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sesa-audio-separation_amd"), os.path.join(REPO, "tests")]
from conftest import CONFIGS  # noqa: E402
from sesa import ops  # noqa: E402
from sesa.models import native as nat  # noqa: E402
from sesa.parallel import _runs, _Windows, shard_plan, side_streams  # noqa: E402
from sesa.utils import get_model_from_config  # noqa: E402
from sesa.weights import synth_state_dict  # noqa: E402

dev = torch.device("cuda:0")
GUARD = 1 << 20  # bytes of NaN guard on each side

_orig_ws = nat.NativeModule.workspace


def guarded_ws(self, device, h, batch):
    need = self._fn("workspace_size")(h, batch)
    key = (device.index, torch.cuda.current_stream(device).cuda_stream, "guard")
    ws = self._ws.get(key)
    if ws is None or ws.numel() < need + 2 * GUARD:
        big = torch.full(((need + 2 * GUARD + 3) // 4,), float("nan"), device=device, dtype=torch.float32)
        self._ws[key] = ws = big.view(torch.uint8)
    return ws[GUARD:GUARD + need]


def run(m, c, mix, plan, rows, eb, streams, sync_each=False, guard=False, clone_y=False):
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
    xs, ys, xguards = [], [], []
    for st in pool[1:]:
        st.wait_stream(main)
    pos, gi = lo, 0
    nat.NativeModule.workspace = guarded_ws if guard else _orig_ws
    while pos < hi:
        grp = flat[pos:min(hi, pos + eb)]
        si = gi % len(pool)
        st = pool[si]
        if st is not main and freed[si] is not None:
            st.wait_event(freed[si])
        with torch.cuda.stream(st):
            if xbufs[si] is None or xbufs[si].shape[0] != len(grp):
                if guard:
                    n = len(grp) * n_ch * C
                    g = GUARD // 4
                    big = torch.full((n + 2 * g,), float("nan"), device=dev, dtype=torch.float32)
                    xguards.append(big)
                    xbufs[si] = big[g:g + n].view(len(grp), n_ch, C)
                else:
                    xbufs[si] = torch.empty(len(grp), n_ch, C, device=dev, dtype=torch.float32)
            xbuf = xbufs[si]
            ops.chunk_gather(mix, plan["border"], [g[0] for g in grp], C, out=xbuf)
            xs.append(xbuf.clone())
            y = m(xbuf).reshape(len(grp), rows, C)
            ys.append(y.clone())
        if st is not main:
            main.wait_stream(st)
            y.record_stream(main)
        if clone_y:
            y = y.clone()
        for j, k in _runs(grp):
            ops.ola_accumulate(y[j:k], [g[0] - s0 for g in grp[j:k]], [g[1] for g in grp[j:k]],
                               win.pick(*grp[j][2:]), local, scratch)
        if st is not main:
            freed[si] = torch.cuda.Event()
            freed[si].record(main)
        if sync_each:
            torch.cuda.synchronize()
        pos += len(grp)
        gi += 1
    for st in pool[1:]:
        main.wait_stream(st)
    torch.cuda.synchronize()
    nat.NativeModule.workspace = _orig_ws
    nan_guard = [bool(torch.isnan(t).all()) for t in xguards]
    return local, xs, ys, nan_guard


def report(tag, ref, out):
    lr, xr, yr, _ = ref
    lo, xo, yo, ng = out
    d = (lr - lo).abs().amax(0)
    bad = torch.nonzero(d > 1e-6).flatten()
    print(f"{tag}: local max diff {float(d.max()):.3e}, {bad.numel()} samples"
          + (f" [{int(bad[0])}..{int(bad[-1])}]" if bad.numel() else ""))
    for g, (a, b, p, q) in enumerate(zip(xr, xo, yr, yo)):
        dx = float((a - b).abs().max())
        dy = float((p - q).abs().max())
        nan_y = bool(torch.isnan(q).any())
        if dx or dy or nan_y:
            where = torch.nonzero((p - q).abs().amax(1) > 1e-6)
            print(f"   group {g}: x diff {dx:.3e}  y diff {dy:.3e}  y NaN {nan_y}  "
                  f"(item, sample) first {where[:3].tolist()} last {where[-3:].tolist()}")
    if ng:
        print(f"   input guards still all-NaN: {ng}")


def main():
    m, c = get_model_from_config("mdx23c", os.path.join(CONFIGS, "config_mdx23c_small.yaml"))
    m.load_state_dict(synth_state_dict(m, affine="random"), strict=True)
    rng = np.random.default_rng(2)
    L = 400000
    mix = torch.from_numpy((0.1 * rng.standard_normal((2, L))).astype(np.float32)).to(dev)
    plan = shard_plan(c, L, 1)
    rows = 4
    eb = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    A = run(m, c, mix, plan, rows, eb, 1)
    A2 = run(m, c, mix, plan, rows, eb, 1)
    report("A2 streams=1 again", A, A2)
    for rep in range(3):
        report(f"B streams=2 (rep {rep})", A, run(m, c, mix, plan, rows, eb, 2))
    report("C streams=2, sync each group", A, run(m, c, mix, plan, rows, eb, 2, sync_each=True))
    report("D streams=2, NaN guards", A, run(m, c, mix, plan, rows, eb, 2, guard=True))
    report("E streams=2, y cloned before OLA", A, run(m, c, mix, plan, rows, eb, 2, clone_y=True))
    report("F streams=3", A, run(m, c, mix, plan, rows, eb, 3))
    # two forwards of the same input at once, many times
    x = torch.from_numpy((0.1 * rng.standard_normal((eb, 2, plan["chunk"]))).astype(np.float32)).to(dev)
    y0 = m(x).clone()
    side = side_streams(dev, 1)[0]
    worst = 0.0
    for _ in range(10):
        side.wait_stream(torch.cuda.current_stream(dev))
        ya = m(x)
        with torch.cuda.stream(side):
            yb = m(x)
        torch.cuda.synchronize()
        worst = max(worst, float((ya - y0).abs().max()), float((yb - y0).abs().max()))
    print(f"G concurrent identical forwards x10: max diff vs single {worst:.3e}")


if __name__ == "__main__":
    main()
