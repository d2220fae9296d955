"""Golden fixture for the GUI registry's conf_edit / get_model_chunk_size (reference model.py).

Run here (not on the GPU box):  python tests/golden/make_golden_registry.py

Imports /root/reference/model.py (needs only yaml / json / re / shutil; ``requests`` is imported
lazily by its download functions, which are never called) and runs the REAL ``conf_edit`` on a set
of input YAML texts in a temporary CHECKPOINT_DIR, recording the edited text (or the exception
type) -> tests/golden/conf_edit.json.  The inputs are synthetic configs shaped like the released
ones (the real YAMLs are fetched at run time and are not in the container).
"""
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))

CASES = [
    ("mdx23c_like", "audio:\n  chunk_size: 261120\n  dim_f: 4096\n  hop_length: 1024\n"
                    "training:\n  instruments:\n  - vocals\n  - other\n  target_instrument: null\n  use_amp: false\n"
                    "inference:\n  batch_size: 1\n  dim_t: 256\n  num_overlap: 2\n", 4),
    ("batch4", "audio:\n  chunk_size: 352800\ninference:\n  batch_size: 4\n  num_overlap: 2\n", 8),
    ("toplevel_use_amp", "use_amp: false\ntraining:\n  use_amp: false\ninference:\n  num_overlap: 2\n", 2),
    ("no_sections", "model:\n  dim: 384\n  depth: 6\n", 4),
    ("url_and_tab", "audio:\n  chunk_size: 485100\nmodel:\n\turl: https://example.org/x.ckpt\n"
                    "\tpath: C:\\models\\x\n\tname: 'q:uoted'\ninference:\n  batch_size: 1\n", 3),
    ("url_only", "model:\n\turl: https://example.org/x.ckpt\n\tname: 'q:uoted'\n\tnote: a \"b\" c:d\n"
                 "inference:\n  batch_size: 1\n", 3),
    ("mixed_tab_indent", "model:\n\turl: https://example.org/x.ckpt\n  path: C:\\m\ninference:\n  batch_size: 1\n", 3),
    ("tuple_tag", "model:\n  freqs_per_bands: !!python/tuple\n  - 2\n  - 2\ninference:\n  batch_size: 1\n", 4),
    ("html", "<!DOCTYPE html>\n<html><body>not yaml</body></html>\n", 4),
    ("broken", "audio:\n  chunk_size: [1, 2\ninference: {\n", 4),
]


def main():
    sys.path.insert(0, "/root/reference")
    import model as ref   # /root/reference/model.py
    out = []
    with tempfile.TemporaryDirectory() as d:
        ref.CHECKPOINT_DIR = d
        for tag, text, overlap in CASES:
            p = os.path.join(d, f"config_{tag}.yaml")
            with open(p, "w", encoding="utf-8") as f:
                f.write(text)
            rec = {"tag": tag, "input": text, "overlap": overlap}
            try:
                ref.conf_edit(p, 0, overlap)
                rec["error"] = None
            except Exception as e:  # noqa: BLE001 -- record the reference's failure type
                rec["error"] = type(e).__name__
            with open(p, encoding="utf-8") as f:
                rec["output"] = f.read()
            rec["backup_left"] = os.path.exists(p + ".backup")
            out.append(rec)
    with open(os.path.join(HERE, "conf_edit.json"), "w", encoding="utf-8") as f:
        json.dump(out, f, indent=1)
    print(f"{len(out)} cases")


if __name__ == "__main__":
    main()
