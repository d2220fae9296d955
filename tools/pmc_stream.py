"""HBM counter bytes of the streaming kernel classes (STFT / iSTFT / chunk gather + OLA) over ONE bench step,
from two rocprofv3 PMC passes (FETCH_SIZE, then WRITE_SIZE in a separate pass; gfx950: FETCH_SIZE doubled,
MI355X_MICROARCH.md §HBM) -- north_star's "rocprof HBM GB/s on the STFT / overlap-add".

usage: python tools/pmc_stream.py <fetch_dir> <write_dir> <model> <precision> <out_dir>
Writes <out_dir>/pmc_{stft,istft,ola}.json: counter bytes per step and per kernel, stamped with the sha of the
class's sources (bench.py KSRC), the workload (model, precision) and $GIT_SHA; bench.py divides the per-step
bytes by the class's live event time to report counter GB/s beside the algorithmic figure.
"""
import importlib.util
import json
import os
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from pmc_traffic import read_counter  # noqa: E402

CLASSES = {"stft": ("stft_kernel", "bsr_stft_kernel", "scn_stft_kernel", "htd_stft"),
           "istft": ("istft_frames_kernel", "istft_ola_kernel", "bsr_istft", "scn_istft", "htd_istft"),
           "ola": ("chunk_gather", "ola_accumulate_kernel", "ola_finalize_kernel")}


def main(fetch_dir, write_dir, model, precision, out_dir):
    spec = importlib.util.spec_from_file_location("bench", os.path.join(HERE, "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    f, fn = read_counter(fetch_dir, "FETCH_SIZE")
    w, wn = read_counter(write_dir, "WRITE_SIZE")
    for kc, subs in CLASSES.items():
        def pick(vals, names):
            per = defaultdict(lambda: [0, 0.0])
            for k, v in vals.items():
                nm = names[k]
                s = next((s for s in subs if s in nm), None)
                if s is not None and not (kc == "stft" and "istft" in nm):
                    per[s][0] += 1
                    per[s][1] += v
            return per
        pf, pw = pick(f, fn), pick(w, wn)
        if not pf:
            continue
        fetch = sum(v[1] for v in pf.values()) * 2 * 1024
        write = sum(v[1] for v in pw.values()) * 1024
        res = {"kernel_class": kc, "model": model, "precision": precision, "steps": 1,
               "hbm_bytes_per_step": round(fetch + write), "fetch_bytes_per_step": round(fetch),
               "write_bytes_per_step": round(write),
               "per_kernel": {s: {"dispatches": pf[s][0], "fetch_bytes": round(pf[s][1] * 2048),
                                  "write_bytes": round(pw.get(s, [0, 0.0])[1] * 1024)} for s in pf},
               "correction": "fetch bytes = 2 * FETCH_SIZE KiB * 1024 (gfx950 counts half of wide coalesced reads), "
                             "write bytes = WRITE_SIZE KiB * 1024; separate --pmc passes",
               "src_sha16": bench.kernel_sources_sha16(kc), "git_sha": os.environ.get("GIT_SHA", "unknown")}
        print(json.dumps(res, indent=1))
        with open(os.path.join(out_dir, f"pmc_{kc}.json"), "w") as fo:
            json.dump(res, fo, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:6])
