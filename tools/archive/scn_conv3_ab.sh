#!/bin/bash
# SCNet 3x3 convs on the MFMA conv-mode GEMM: SCNet parity suite + same-box A/B of the SCNet bench and the
# ensemble (SESA_SCN_CONV3_VALU=1: the exact-fp32 VALU kernel).
set -e
O=gpurun_out/scn3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[scn3] $(date +%T) tests"
timeout -k 10 500 python -u -m pytest tests/test_scnet.py tests/test_ensemble_models.py -m gpu -x -v --timeout 200 --timeout-method thread -s > $O/test.log 2>&1
for v in M:0 V:1 Mb:0 Vb:1; do
  n=${v%%:*}; m=${v##*:}
  echo "[scn3] $(date +%T) bench $n ($m)"
  SESA_SCN_CONV3_VALU=$m timeout -k 10 300 python bench.py --model scnet --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err
done
echo "[scn3] $(date +%T) done"
