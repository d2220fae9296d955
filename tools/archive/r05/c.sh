#!/bin/bash
# Round 5 lease C: workspace hygiene (tools/ws_guard.py), configs[4] blend parity scan, and bench lines of every model
# with the per-class rooflines (algorithmic bytes per launch, intensity-picked bound, per-launch floor fraction).
set -e
O=gpurun_out/r05c
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05c] $(date +%T) ws_guard"
timeout -k 10 400 python -u tools/ws_guard.py > $O/ws_guard.txt 2>&1
echo "[r05c] $(date +%T) ens scan"
timeout -k 10 400 python -u tools/ens_parity_scan.py > $O/ens_scan.txt 2>&1
for m in mdx23c bs_roformer htdemucs scnet; do
  echo "[r05c] $(date +%T) bench $m"
  timeout -k 10 300 python bench.py --model $m --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$m.json 2> $O/bench_$m.err
done
echo "[r05c] $(date +%T) done"
