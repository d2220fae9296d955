#!/bin/bash
# Round 5 lease Q: persistent rewrite-conv workgroups (SESA_HTD_RW_PERS=1: the next tile's first chunk prefetched
# under the current tile's last) vs one tile per workgroup -- HTDemucs GPU tests with it on, same-box benches.
set -e
O=gpurun_out/r05q
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05q] $(date +%T) tests (persistent)"
SESA_HTD_RW_PERS=1 timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/tests.txt 2>&1
b() {
  echo "[r05q] $(date +%T) bench $1"
  timeout -k 10 400 python bench.py $2 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
b base "--model htdemucs --steps 3 --warmup 1 --no-parity"
SESA_HTD_RW_PERS=1 b pers "--model htdemucs --steps 3 --warmup 1"
b base2 "--model htdemucs --steps 3 --warmup 1 --no-parity"
SESA_HTD_RW_PERS=1 b pers2 "--model htdemucs --steps 3 --warmup 1 --no-parity"
echo "[r05q] $(date +%T) done"
