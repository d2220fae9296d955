#!/bin/bash
# Round 4: conv3x3 phase-order A/B (conv_bench f16), BS-/Mel-Band-Roformer fp16 attention + out-projection parity,
# BS-Roformer fp16 vs bf16x3 bench (same box, no CPU leg).
set -e
O=gpurun_out/r04b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04b] $(date +%T) conv_bench f16"
timeout -k 10 300 ./tools/conv_bench 57 f16 > $O/conv_f16.txt 2>&1
echo "[r04b] $(date +%T) bsr parity"
timeout -k 10 600 python -u -m pytest tests/test_bsr.py tests/test_amp_precision.py tests/test_gpu_parity.py -v -s --timeout 300 \
  --timeout-method thread -k "fp16 or full_chunk or small or roformer or large or side_streams" > $O/parity.txt 2>&1 || rc=$?
if [ "${rc:-0}" != 0 ]; then echo "[r04b] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
run() {
  echo "[r04b] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py --model bs_roformer --precision $3 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
run bsr_fp16 fp=1 fp16
run bsr_bf16x3 fp=1 bf16x3
run bsr_fp16b fp=1 fp16
mrun() {
  echo "[r04b] $(date +%T) mdx $1"
  timeout -k 10 300 env $2 python bench.py --precision $3 --steps 10 --warmup 2 --no-cpu-baseline > $O/mdx_$1.json 2> $O/mdx_$1.err
}
mrun mix_ord1 SESA_CONV_ORD=1 fp16mix
mrun mix_ord0 SESA_CONV_ORD=0 fp16mix
mrun fp16_ord1 SESA_CONV_ORD=1 fp16
mrun fp16_ord0 SESA_CONV_ORD=0 fp16
mrun mix_ord1b SESA_CONV_ORD=1 fp16mix
echo "[r04b] $(date +%T) done"
