#!/bin/bash
# HTDemucs 64-column conv tiles: parity (tests/test_htdemucs.py) + same-box A/B of the configs[3] bench
# (SESA_HCONV_BN64=1 default: N <= 64; =0: 128-column tiles everywhere; =all: also N = 64 mod 128).
set -e
O=gpurun_out/bn64
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[bn64] $(date +%T) tests"
timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py -m gpu -x -v --timeout 200 --timeout-method thread -s > $O/test.log 2>&1
for v in B1:1 B0:0 B2:all B1b:1 B0b:0 B2b:all; do
  n=${v%%:*}; m=${v##*:}
  echo "[bn64] $(date +%T) bench $n ($m)"
  SESA_HCONV_BN64=$m timeout -k 10 300 python bench.py --model htdemucs --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err
done
echo "[bn64] $(date +%T) done"
