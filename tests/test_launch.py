"""``bench.py --gpus N`` from a plain command line: the launcher
(sesa/launch.py) starts N rank processes under torch.distributed.run as a child of a parent that has
not touched HIP; each rank reads its rank / world from the environment and refuses a world size other
than --gpus.  CPU: the same launcher drives tests/_launch_worker.py (gloo, StandIn model, the
chunk-shard plan + all_gather + seam assembly of sesa/parallel.py) and the result must equal the
world-1 result; bench.py itself must refuse a mismatched world before any device work."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import REPO

WORKER = os.path.join(REPO, "tests", "_launch_worker.py")


def _world1(mode):
    import test_parallel_gloo as t
    from sesa.parallel import demix_sharded
    cfg = t._demucs_cfg() if mode == "demucs" else t._cfg(2)
    return demix_sharded(cfg, t.StandIn(), torch.from_numpy(t._mix()), rank=0, world=1, local_fn=t.cpu_local,
                         finalize_fn=t.cpu_finalize, counter_fn=t.make_cpu_counter(cfg), mode=mode).numpy()


def test_needs_spawn_rules():
    from sesa.launch import needs_spawn
    assert needs_spawn(2, {}) and needs_spawn(8, {"RANK": "0"})
    assert not needs_spawn(1, {}) and not needs_spawn(2, {"WORLD_SIZE": "2"})


@pytest.mark.parametrize("world,mode", [(2, "generic"), (3, "demucs")])
def test_spawned_world_matches_world1(tmp_path, world, mode):
    from sesa.launch import spawn_world
    out = str(tmp_path / "est.npy")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    rc = subprocess.run([sys.executable, "-c",
                         "import sys; sys.path.insert(0, %r); from sesa.launch import spawn_world; "
                         "sys.exit(spawn_world(%d, %r, ['--gpus', '%d', '--out', %r, '--mode', %r]))"
                         % (os.path.join(REPO, "sesa-audio-separation_amd"), world, WORKER, world, out, mode)],
                        env=env, timeout=600).returncode
    assert rc == 0
    est = np.load(out)
    meta = json.load(open(out + ".json"))
    assert meta["world"] == world and len(meta["ranges"]) == world
    ref = _world1(mode)
    assert est.shape == ref.shape
    # seams summed per rank: fp32 regrouping only
    assert np.abs(est - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max())
    assert spawn_world is not None


def test_bench_refuses_mismatched_world():
    """torchrun world 1 but --gpus 2: bench.py exits 3 before touching the device."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 3 and "WORLD_SIZE=1" in r.stderr


def test_worker_refuses_mismatched_world(tmp_path):
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, WORKER, "--gpus", "3", "--out", str(tmp_path / "x.npy")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 3
