#!/bin/bash
# Winograd F(2,3) TFC convs (opt-in): MDX23C parity suite incl. the Winograd goldens, the per-level
# micro-benchmark with ablations, and a same-box A/B of the headline bench (default = direct kernels;
# SESA_CONV_WINO=1: Winograd at levels 1-3; all: levels 0-3).
set -e
O=gpurun_out/wino
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[wino] $(date +%T) parity"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -s > $O/test.log 2>&1
echo "[wino] $(date +%T) conv_bench"
timeout -k 10 300 ./tools/conv_bench 57 wino > $O/conv_bench.txt 2>&1
for v in W0:0 W1:1 W2:all W0b:0; do
  n=${v%%:*}; m=${v##*:}
  echo "[wino] $(date +%T) bench $n ($m)"
  SESA_CONV_WINO=$m timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err
done
echo "[wino] $(date +%T) done"
