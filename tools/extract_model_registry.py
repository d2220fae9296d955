"""Generate sesa-audio-separation_amd/sesa/model_registry.json from the reference GUI registry.

Run here (the reference tree is not on the GPU box):  python tools/extract_model_registry.py

The reference's ``MODEL_CONFIGS`` (/root/reference/model.py:533-1767) is a literal dict whose paths
are ``os.path.join(CHECKPOINT_DIR, <file>)`` calls.  This script evaluates ONLY that assignment
(found with ``ast``; no other reference code runs) with CHECKPOINT_DIR / BASE_DIR bound to
placeholders, and records per entry the category, display name, model_type, config / checkpoint
FILE NAMES, download URLs, ``custom_model_url`` and ``needs_conf_edit`` -- the data the registry
(sesa/registry.py) needs.  The JSON is data, not code.
"""
import ast
import json
import os

REF = "/root/reference/model.py"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "sesa-audio-separation_amd", "sesa", "model_registry.json")
CKPT = "<CHECKPOINT_DIR>"


def main():
    with open(REF, encoding="utf-8") as f:
        tree = ast.parse(f.read())
    node = next(n for n in tree.body if isinstance(n, ast.Assign)
                and any(isinstance(t, ast.Name) and t.id == "MODEL_CONFIGS" for t in n.targets))
    code = compile(ast.Module(body=[node], type_ignores=[]), REF, "exec")
    ns = {"os": os, "CHECKPOINT_DIR": CKPT, "BASE_DIR": "<BASE_DIR>"}
    exec(code, ns)  # the dict literal only
    out = []
    for category, entries in ns["MODEL_CONFIGS"].items():
        for name, e in entries.items():
            def base(p):
                assert p.startswith(CKPT), p
                return os.path.basename(p)
            urls = []
            for u in e["download_urls"]:
                urls.append(list(u) if isinstance(u, tuple) else u)
            out.append({"category": category, "name": name, "model_type": e["model_type"],
                        "config_file": base(e["config_path"]), "checkpoint_file": base(e["start_check_point"]),
                        "download_urls": urls, "custom_model_url": e.get("custom_model_url"),
                        "needs_conf_edit": bool(e["needs_conf_edit"])})
    with open(OUT, "w", encoding="utf-8") as f:
        json.dump({"source": "reference model.py:533-1767 MODEL_CONFIGS", "entries": out}, f, indent=1,
                  ensure_ascii=False)
    print(f"{len(out)} entries -> {OUT}")


if __name__ == "__main__":
    main()
