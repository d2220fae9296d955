"""Rank program for tests/test_launch.py: started N times by sesa.launch.spawn_world (the launcher
bench.py uses for ``--gpus N``), it joins a gloo group from the torchrun environment, refuses a
world size that differs from --gpus (as bench.py does), and runs the chunk-shard path
(sesa.parallel.demix_sharded: shard plan, span all_gather, seam assembly) with the StandIn model and
the oracle OLA of tests/test_parallel_gloo.py.  Rank 0 saves the estimate and the plan's ranges."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import conftest  # noqa: E402,F401  (repo + package on sys.path)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--mode", default="generic")
    args = ap.parse_args()
    from sesa.launch import world_from_env
    rank, local_rank, world = world_from_env()
    if world != args.gpus:
        print(f"world {world} != --gpus {args.gpus}", file=sys.stderr)
        return 3
    dist.init_process_group("gloo")
    try:
        if dist.get_world_size() != args.gpus:
            return 3
        import test_parallel_gloo as t
        from sesa.parallel import demix_sharded, shard_plan
        cfg = t._demucs_cfg() if args.mode == "demucs" else t._cfg(2)
        est = demix_sharded(cfg, t.StandIn(), torch.from_numpy(t._mix()), local_fn=t.cpu_local,
                            finalize_fn=t.cpu_finalize, counter_fn=t.make_cpu_counter(cfg), mode=args.mode)
        if rank == 0:
            np.save(args.out, est.numpy())
            with open(args.out + ".json", "w") as f:
                json.dump({"world": dist.get_world_size(), "local_rank": local_rank,
                           "ranges": shard_plan(cfg, t.L_TRACK, world, args.mode)["ranges"]}, f)
    finally:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
