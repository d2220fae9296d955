#!/bin/bash
# Round 4: HTDemucs fp16mix with fp16 q / k / v planes into the attention (self + cross): parity and bench;
# MDX23C encoder-level-0 TDF in fp16 (SESA_TDF_PLAN=1333111111111111): parity on the four fixtures + A/B.
set -e
O=gpurun_out/r04l
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04l] $(date +%T) parity"
timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py -v -s --timeout 300 --timeout-method thread \
  -k "full_segment or small_matches" > $O/parity_htd.txt 2>&1 || rc=$?
if [ "${rc:-0}" != 0 ]; then echo "[r04l] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
SESA_TDF_PLAN=1333111111111111 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 300 \
  --timeout-method thread -k "levels and fp16mix" > $O/parity_tdf0.txt 2>&1 || rc=$?
if [ "${rc:-0}" != 0 ]; then echo "[r04l] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
run() {
  echo "[r04l] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py $3 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
run htd fp=1 "--model htdemucs --steps 1 --warmup 1"
run mdx fp=1 "--steps 6 --warmup 1"
run mdx_tdf0 SESA_TDF_PLAN=1333111111111111 "--steps 6 --warmup 1"
run mdx_b fp=1 "--steps 6 --warmup 1"
run mdx_tdf0b SESA_TDF_PLAN=1333111111111111 "--steps 6 --warmup 1"
echo "[r04l] $(date +%T) done"
