#!/bin/bash
# fp16 TFC-conv precisions: GPU parity (the new tests + the existing MDX23C ones) and a same-box bench A/B
# (bf16x3 / fp16w2 / fp16 / bf16x3 again) of the configs[1] headline.
set -e
O=gpurun_out/f16
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[f16] $(date +%T) tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "fp16_conv or full_chunk or small or stress" > $O/gputest.log 2>&1
for P in bf16x3 fp16w2 fp16 bf16x3b; do
  echo "[f16] $(date +%T) bench $P"
  timeout -k 10 300 python bench.py --precision ${P%b} --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$P.json 2> $O/bench_$P.err
done
echo "[f16] $(date +%T) done"
