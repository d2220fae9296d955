#!/bin/bash
# Winograd F(2,3) TFC convs: MDX23C parity suite, then a same-box A/B of the headline bench
# (SESA_CONV_WINO=0: direct conv3x3_db everywhere; default: Winograd at levels 1-3; all: levels 0-3).
set -e
O=gpurun_out/wino
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[wino] $(date +%T) parity"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -s > $O/test.log 2>&1
for v in W1:1 W0:0 W2:all W1b:1 W2b:all W0b:0; do
  n=${v%%:*}; m=${v##*:}
  echo "[wino] $(date +%T) bench $n ($m)"
  SESA_CONV_WINO=$m timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err
done
echo "[wino] $(date +%T) done"
