#!/bin/bash
# Round 5 lease G: one-GPU rehearsals of rank 0's share of 2/4/8-rank runs (bench.py --rank-share) for MDX23C and
# HTDemucs, and HTDemucs with the per-h DConv kernel selection.
set -e
O=gpurun_out/r05g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
b() {
  echo "[r05g] $(date +%T) $1"
  timeout -k 10 400 python bench.py $2 --no-cpu-baseline --no-parity > $O/bench_$1.json 2> $O/bench_$1.err
}
b htd "--model htdemucs --steps 3 --warmup 1"
for w in 2 4 8; do b mdx_share$w "--rank-share $w --steps 5 --warmup 1"; done
for w in 2 4 8; do b htd_share$w "--model htdemucs --rank-share $w --steps 3 --warmup 1"; done
b mdx "--steps 5 --warmup 1"
echo "[r05g] $(date +%T) done"
