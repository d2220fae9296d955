"""The GUI process boundary: the launch targets the reference GUI spawns, run as
fresh child processes exactly as processing.py does.

* separation: processing.py:250-252 launches ``inference_pytorch.INFERENCE_PATH`` (falling back to
  inference.py) with the argv built at :266-304 (``--export_format "wav FLOAT"``, the optimized-backend
  flags), cwd = BASE_DIR, and reads ``[SESA_PROGRESS]`` lines from the child's stdout line by line
  (:323-363); a non-zero exit is an error (:372-375).  The stems are checked against what the real
  reference run_folder_pytorch_optimized wrote for the same flags (tests/golden/cli_flow.npz, case
  ``tta_demud_instr``: TTA + demud phase remix + extract_instrumental, WAV FLOAT).
* ensemble: processing.py:735 runs ``python ensemble.py --files ... --type ... --output ...`` from the
  base directory and parses the same progress protocol; exit 0 / 1 (ensemble.py:409-441).

The children are started with ``subprocess.Popen`` (never an exec of the test process)."""
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

from conftest import PKG_ROOT, rms

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_cli_flow import RMS_GATE, _cases, _setup  # noqa: E402

from oracle import ensemble as oe  # noqa: E402


def _gui_run(cmd_parts, cwd, timeout=300):
    """processing.py:306-375: Popen with piped text stdout / stderr, stdout read line by line for the
    progress protocol, then the exit code.  (stderr is drained on a thread so a chatty child cannot
    block on a full pipe while the parent is still reading stdout.)"""
    proc = subprocess.Popen(cmd_parts, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                            bufsize=1, universal_newlines=True)
    err = []
    t = threading.Thread(target=lambda: err.append(proc.stderr.read()), daemon=True)
    t.start()
    progress, other = [], []
    timer = threading.Timer(timeout, proc.kill)
    timer.start()
    try:
        for line in proc.stdout:
            s = line.strip()
            if s.startswith("[SESA_PROGRESS]"):
                pct = float(s.replace("[SESA_PROGRESS]", "").strip() or 0)
                progress.append(min(max(pct, 0), 100))
            elif s:
                other.append(s)
        proc.wait()
    finally:
        timer.cancel()
    t.join(timeout=10)
    return proc.returncode, progress, other, "".join(err)


def _gui_separation_argv(script, cfg_path, ckpt, inp, out, use_tta, demud, extract):
    """processing.py:266-304 (output_format 'wav', AMP off, TF32 + cuDNN benchmark on as the GUI
    defaults pass them)."""
    cmd = ["python", script, "--model_type", "mdx23c", "--config_path", str(cfg_path),
           "--start_check_point", str(ckpt), "--input_folder", str(inp), "--store_dir", str(out),
           "--chunk_size", "261120", "--overlap", "4", "--export_format", "wav FLOAT",
           "--optimize_mode", "channels_last", "--enable_tf32", "--enable_cudnn_benchmark"]
    if extract:
        cmd.append("--extract_instrumental")
    if use_tta:
        cmd.append("--use_tta")
    if demud:
        cmd.append("--demud_phaseremix_inst")
    cmd[0] = sys.executable   # "python" on the GUI's PATH == this interpreter
    return cmd


def test_launch_targets_exist_and_import():
    """processing.py:250 does ``from inference_pytorch import INFERENCE_PATH`` with BASE_DIR on the
    path; both scripts answer --help with exit 0 in a fresh interpreter."""
    for name in ("inference.py", "inference_pytorch.py", "ensemble.py"):
        assert os.path.isfile(os.path.join(PKG_ROOT, name)), name
    code = "import inference_pytorch as ip, os; print(ip.INFERENCE_PATH)"
    r = subprocess.run([sys.executable, "-c", code], cwd=PKG_ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip() == os.path.join(PKG_ROOT, "inference_pytorch.py")
    for name in ("inference_pytorch.py", "ensemble.py"):
        r = subprocess.run([sys.executable, name, "--help"], cwd=PKG_ROOT, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0 and "usage" in r.stdout.lower(), (name, r.stderr[-2000:])


def test_ensemble_child_exit_code_on_bad_input(tmp_path):
    """ensemble.py exits 1 (not a traceback / 0) when validation fails -- here a single input file."""
    from sesa.audio_io import write_audio
    p = tmp_path / "one.wav"
    write_audio(str(p), np.zeros((100, 2), np.float32), 44100, subtype="FLOAT")
    rc, prog, _, err = _gui_run([sys.executable, "ensemble.py", "--files", str(p), "--type", "avg_wave",
                                 "--output", str(tmp_path / "o.wav")], PKG_ROOT)
    assert rc == 1 and prog == [], err[-2000:]


@pytest.mark.gpu
def test_gui_separation_child_process_matches_reference(tmp_path):
    from sesa.audio_io import read_any
    metas, g = _cases()
    case = next(c for c in metas if c["tag"] == "tta_demud_instr")
    cfg_path, ckpt, inp = _setup(tmp_path, case)
    out = tmp_path / "out"
    fl = case["flags"]
    cmd = _gui_separation_argv(os.path.join(PKG_ROOT, "inference_pytorch.py"), cfg_path, ckpt, inp, out,
                               fl.get("use_tta", False), fl.get("demud_phaseremix_inst", False),
                               fl.get("extract_instrumental", False))
    rc, prog, other, err = _gui_run(cmd, PKG_ROOT)
    assert rc == 0, (other[-20:], err[-3000:])
    # the progress values the GUI parsed (clamped to [0, 100] as processing.py:347 does -- the reference
    # prints values past 100 on the TTA passes) are the reference's lines, in order
    assert prog == [min(max(float(s.replace("[SESA_PROGRESS]", "")), 0), 100) for s in case["progress"]]
    assert sorted(os.listdir(out)) == sorted(case["outputs"])
    for fn, o in case["outputs"].items():
        got, sr = read_any(str(out / fn))
        ref = g[o["key"]]
        assert sr == o["sr"] and got.shape == ref.T.shape and o["subtype"] == "FLOAT"
        err_rms = rms(got.T, ref)
        print(f"gui child {fn}: rms {err_rms:.3e}")
        assert err_rms <= RMS_GATE


@pytest.mark.gpu
def test_gui_separation_child_reports_failure(tmp_path):
    """A missing config makes the child exit non-zero with the reason on stderr (processing.py:372-375
    raises CalledProcessError with it)."""
    out = tmp_path / "out"
    (tmp_path / "in").mkdir()
    cmd = _gui_separation_argv(os.path.join(PKG_ROOT, "inference_pytorch.py"), tmp_path / "missing.yaml",
                               tmp_path / "none.ckpt", tmp_path / "in", out, False, False, False)
    rc, prog, _, err = _gui_run(cmd, PKG_ROOT)
    assert rc != 0 and err.strip()


@pytest.mark.gpu
def test_gui_ensemble_child_process(tmp_path):
    from sesa.audio_io import quantize_pcm, read_wav, write_audio
    rng = np.random.default_rng(11)
    d = tmp_path / "stems dir"          # a space in the path: the reference's PCM_16 re-encode quirk
    d.mkdir()
    files = []
    for i in range(3):
        x = (0.1 * rng.standard_normal((2, 70000 - 500 * i))).astype(np.float32)
        p = d / f"m{i}_vocals.wav"
        write_audio(str(p), x.T, 44100, subtype="PCM_24")
        files.append(str(p))
    out = tmp_path / "ens.wav"
    cmd = [sys.executable, "ensemble.py", "--files", *files, "--type", "avg_wave", "--output", str(out),
           "--weights", "1.0", "2.0", "1.0"]
    rc, prog, other, err = _gui_run(cmd, PKG_ROOT)
    assert rc == 0, (other[-20:], err[-3000:])
    assert prog and prog[-1] == 100 and prog == sorted(prog)
    y, sr = read_wav(str(out))
    ins = [read_wav(f)[0] for f in files]
    n = min(a.shape[1] for a in ins)
    # special-character paths are re-encoded at soundfile's default PCM_16 first (ensemble.py:70-79)
    ins = np.stack([quantize_pcm(a[:, :n], 16) / 32768.0 for a in ins]).astype(np.float64)
    exp = oe.blend(ins, "avg_wave", [1.0, 2.0, 1.0])
    exp_q = quantize_pcm(exp.astype(np.float32), 24) / 8388608.0
    assert sr == 44100 and y.shape == (2, n)
    assert np.abs(y - exp_q).max() <= 1.0 / 8388608 + 1e-9
