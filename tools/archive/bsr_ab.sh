#!/bin/bash
# Same-box A/B of the BS-Roformer attention operand form (SESA_BSR_QKV_PLANES=1 default: q / k / v written as
# bf16 planes by the projection epilogue; =0: fp32 rows split by attn_kernel).
set -e
O=gpurun_out/bsrab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in P1:1 P0:0 P1b:1 P0b:0; do
  n=${v%%:*}; m=${v##*:}
  echo "[bsrab] $(date +%T) $n"
  SESA_BSR_QKV_PLANES=$m timeout -k 10 300 python bench.py --model bs_roformer --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err
done
echo "[bsrab] $(date +%T) done"
