"""GUI model registry (reference model.py:135-227, :294-421, :533-1880), offline.

conf_edit is checked text-for-text against the REAL reference conf_edit run on the same inputs
(tests/golden/conf_edit.json, tests/golden/make_golden_registry.py).  The registry table equals the
reference MODEL_CONFIGS (121 entries; tools/extract_model_registry.py).  No network: missing
checkpoint / config files raise instead of downloading.
"""
import importlib
import json
import os

import pytest
import yaml

from conftest import GOLDEN


@pytest.fixture
def reg(tmp_path, monkeypatch):
    monkeypatch.setenv("SESA_CHECKPOINT_DIR", str(tmp_path / "ckpts"))
    monkeypatch.setenv("SESA_CUSTOM_MODELS", str(tmp_path / "assets" / "custom_models.json"))
    os.makedirs(tmp_path / "ckpts")
    import sesa.registry as r
    r = importlib.reload(r)
    yield r
    monkeypatch.delenv("SESA_CHECKPOINT_DIR")
    monkeypatch.delenv("SESA_CUSTOM_MODELS")
    importlib.reload(r)


def test_table_matches_reference(reg):
    names = reg.get_model_config()
    assert sum(len(c) for c in reg.MODEL_CONFIGS.values()) == 121   # one display name is in two categories
    assert len(names) == 120
    assert reg.get_model_config.keys() == names
    counts = {}
    for cat in reg.MODEL_CONFIGS.values():
        for e in cat.values():
            counts[e["model_type"]] = counts.get(e["model_type"], 0) + 1
    assert counts["mel_band_roformer"] == 83 and counts["bs_roformer"] == 22 and counts["mdx23c"] == 4
    assert counts["scnet"] == 3
    e = reg.MODEL_CONFIGS["Vocal Models"]["VOCALS-InstVocHQ"]
    assert e["model_type"] == "mdx23c" and e["needs_conf_edit"] is False
    assert os.path.basename(e["config_path"]) == "config_vocals_mdx23c.yaml"
    assert os.path.basename(e["start_check_point"]) == "model_vocals_mdx23c_sdr_10.17.ckpt"


@pytest.mark.parametrize("case", json.load(open(os.path.join(GOLDEN, "conf_edit.json"))),
                         ids=lambda c: c["tag"])
def test_conf_edit_matches_reference(reg, case):
    p = os.path.join(reg.CHECKPOINT_DIR, f"config_{case['tag']}.yaml")
    with open(p, "w", encoding="utf-8") as f:
        f.write(case["input"])
    err = None
    try:
        reg.conf_edit(p, 0, case["overlap"])
    except Exception as e:  # noqa: BLE001
        err = type(e).__name__
    assert err == case["error"]
    with open(p, encoding="utf-8") as f:
        assert f.read() == case["output"]
    assert os.path.exists(p + ".backup") == case["backup_left"]


def test_get_model_config_offline(reg):
    name = "VOCALS-InstVocHQ"
    with pytest.raises(FileNotFoundError, match="config_vocals_mdx23c.yaml"):
        reg.get_model_config(name, 261120, 4)
    d = reg.CHECKPOINT_DIR
    cfg_text = "audio:\n  chunk_size: 261120\ninference:\n  batch_size: 1\n  num_overlap: 2\n"
    with open(os.path.join(d, "config_vocals_mdx23c.yaml"), "w") as f:
        f.write(cfg_text)
    open(os.path.join(d, "model_vocals_mdx23c_sdr_10.17.ckpt"), "wb").close()
    mt, cp, ck = reg.get_model_config(name, 261120, 4)
    assert (mt, os.path.basename(cp), os.path.basename(ck)) == (
        "mdx23c", "config_vocals_mdx23c.yaml", "model_vocals_mdx23c_sdr_10.17.ckpt")
    with open(cp) as f:                                   # needs_conf_edit False: untouched
        assert f.read() == cfg_text
    assert reg.get_model_chunk_size(name) == 261120
    assert reg.get_model_config("no such model") == ("", "", "")


def test_get_model_config_applies_conf_edit(reg):
    name, e = next((n, e) for cat in reg.MODEL_CONFIGS.values() for n, e in cat.items()
                   if e["needs_conf_edit"] and e["model_type"] == "mel_band_roformer" and len(e["download_urls"]) == 2
                   and not e.get("custom_model_url"))
    for u in e["download_urls"]:
        fn = u[1] if isinstance(u, tuple) else os.path.basename(u)
        with open(os.path.join(reg.CHECKPOINT_DIR, fn), "w") as f:
            f.write("audio:\n  chunk_size: 352800\ninference:\n  batch_size: 1\n  num_overlap: 2\n")
    reg.get_model_config(name, 352800, 8)
    with open(e["config_path"]) as f:
        d = yaml.safe_load(f)
    assert d["inference"] == {"batch_size": 2, "num_overlap": 8}
    assert d["training"]["use_amp"] is True and d["audio"]["chunk_size"] == 352800


def test_custom_models(reg):
    ok, msg = reg.add_custom_model("My HT", "auto", "https://huggingface.co/u/r/blob/main/htdemucs_ft.th",
                                   "https://huggingface.co/u/r/blob/main/cfg.yaml")
    assert ok, msg
    c = reg.load_custom_models()["My HT"]
    assert c["model_type"] == "htdemucs" and "/resolve/" in c["checkpoint_url"]
    assert c["config_filename"] == "config_my_ht.yaml"
    assert reg.add_custom_model("My HT", "mdx23c", "a", "b") == (False, "Model 'My HT' already exists")
    assert reg.add_custom_model("X", "foo", "a", "b") == (False, "Unsupported model type: foo")
    assert ("My HT", "htdemucs") in reg.get_custom_models_list()
    assert "My HT" in reg.get_model_config()
    assert "Custom Models" in reg.get_all_model_configs_with_custom()
    assert reg.delete_custom_model("My HT")[0]
    assert reg.load_custom_models() == {}


def test_native_flags(reg):
    assert reg.is_native("mdx23c") and reg.is_native("htdemucs") and not reg.is_native("bandit_v2")
