#!/bin/bash
# Round 4: fp16 token GEMM ring depth (compact fp16 stages, DEPTH 2/3/4) on the BS-Roformer Linear shapes;
# MDX23C with the conv3x3 shortcut on the per-wave DMA ring: parity, then a same-box A/B against the
# LDS-staged shortcut (SESA_CONV_SCR=0) on the configs[1] headline bench.
set -e
O=gpurun_out/r04f
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04f] $(date +%T) tokgemm_bench f16"
timeout -k 10 300 ./tools/tokgemm_bench 198648 f16 > $O/tokgemm_f16.txt 2>&1
echo "[r04f] $(date +%T) parity"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_amp_precision.py -v --timeout 300 \
  --timeout-method thread -k "levels or matrix or mdx23c or fp16 or config0 or full_size" > $O/parity.txt 2>&1 || rc=$?
if [ "${rc:-0}" != 0 ]; then echo "[r04f] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
run() {
  echo "[r04f] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
run ring fp=1
run lds SESA_CONV_SCR=0
run ring_b fp=1
run lds_b SESA_CONV_SCR=0
echo "[r04f] $(date +%T) htdemucs fp16 attention parity"
timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py -v --timeout 300 --timeout-method thread \
  -k "small_matches or full_segment" > $O/parity_htd.txt 2>&1 || rc=$?
if [ "${rc:-0}" != 0 ]; then echo "[r04f] htd parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
for p in fp16mix bf16x3; do
  echo "[r04f] $(date +%T) htdemucs $p"
  timeout -k 10 400 python bench.py --model htdemucs --precision $p --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_htd_$p.json 2> $O/bench_htd_$p.err
done
echo "[r04f] $(date +%T) done"
