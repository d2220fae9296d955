"""Markdown table of the round's bench lines: python tools/numbers_table.py profiles/r04_final_bench_*.json"""
import json
import sys


def main(paths):
    print("| Line | × real-time | dtype | parity (worst fixture RMS) | dominant class: achieved / peak (frac) | "
          "CPU baseline | file |")
    print("|---|---|---|---|---|---|---|")
    for p in paths:
        try:
            d = json.loads(open(p).read().strip().splitlines()[-1])
        except Exception as e:  # noqa: BLE001
            print(f"| {p} | unreadable ({e}) |")
            continue
        r = d.get("roofline") or {}
        cb = d.get("cpu_baseline") or {}
        cpu = f"{cb.get('value', 0):.4g} {cb.get('unit', '')}" if cb else "—"
        name = d.get("config", {}).get("model", "?")
        dom = (f"{r.get('kernel', '?').split(' (')[0]}: {r.get('achieved')} / {r.get('peak')} {r.get('unit', '')} "
               f"({r.get('frac')})")
        print(f"| {name} | {d['value']:.1f} | {d.get('dtype')} | {d.get('parity_rms', 0):.3g} | {dom} | {cpu} | "
              f"`{p}` |")


if __name__ == "__main__":
    main(sys.argv[1:])
