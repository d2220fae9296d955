#!/bin/bash
# BS-Roformer fp16 Linears (SESA_PREC_F16): GPU parity (BSR / Mel-Band tests) and a same-box bench A/B
set -e
O=gpurun_out/bsr16
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[bsr16] $(date +%T) tests"
timeout -k 10 400 python -u -m pytest tests/test_bsr.py -m gpu -x -v --timeout 150 --timeout-method thread > $O/gputest.log 2>&1
for P in bf16x3 fp16 bf16x3b fp16b; do
  echo "[bsr16] $(date +%T) bench $P"
  timeout -k 10 300 python bench.py --model bs_roformer --precision ${P%b} --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$P.json 2> $O/bench_$P.err
done
echo "[bsr16] $(date +%T) done"
