#!/bin/bash
# Round 5 lease R: persistent rewrite-conv workgroups (SESA_HTD_RW_PERS=1: the next tile's first chunk prefetched
# under the current tile's last) and the fused iSTFT frames + overlap-add (SESA_HTD_ISTFT_FUSED=1) vs the defaults --
# HTDemucs GPU tests with both on, same-box benches.
set -e
O=gpurun_out/r05r
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05r] $(date +%T) tests (persistent + fused iSTFT)"
SESA_HTD_RW_PERS=1 SESA_HTD_ISTFT_FUSED=1 timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
b() {
  echo "[r05r] $(date +%T) bench $1"
  timeout -k 10 400 python bench.py $2 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
b base "--model htdemucs --steps 3 --warmup 1 --no-parity"
SESA_HTD_RW_PERS=1 b pers "--model htdemucs --steps 3 --warmup 1"
SESA_HTD_ISTFT_FUSED=1 b fused "--model htdemucs --steps 3 --warmup 1"
SESA_HTD_RW_PERS=1 SESA_HTD_ISTFT_FUSED=1 b both "--model htdemucs --steps 3 --warmup 1 --no-parity"
b base2 "--model htdemucs --steps 3 --warmup 1 --no-parity"
echo "[r05r] $(date +%T) done"
