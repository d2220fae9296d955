#!/bin/bash
# fp16 TFC convs: same-box A/B of the level-0 fused activation (SESA_CONV_FUSED_ACT=0: act_split fp16 plane
# + plain staging) against the default (fused), configs[1] headline bench.
set -e
O=gpurun_out/f16ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  echo "[f16ab] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py --precision $3 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
run fused fp=1 fp16
run unfused SESA_CONV_FUSED_ACT=0 fp16
run fused2 fp=1 fp16
run unfused2 SESA_CONV_FUSED_ACT=0 fp16
run w2_unfused SESA_CONV_FUSED_ACT=0 fp16w2
echo "[f16ab] $(date +%T) done"
