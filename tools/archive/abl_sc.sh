#!/bin/bash
# ablation: fp16 MI4 TFC convs with / without the fused shortcut chunks (SESA_ABL_NO_SC=1 gives wrong stems)
set -e
O=gpurun_out/ablsc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in "base fp=1" "nosc SESA_ABL_NO_SC=1" "base2 fp=1" "nosc2 SESA_ABL_NO_SC=1"; do
  set -- $c
  echo "[abl] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/bench_$1.json 2> $O/bench_$1.err
done
echo "[abl] done"
