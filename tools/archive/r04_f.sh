#!/bin/bash
# Round 4: fp16 token GEMM ring depth (compact fp16 stages, DEPTH 2/3/4) on the BS-Roformer Linear shapes and
# end to end (SESA_TOKGEMM_DEPTH); MDX23C with the conv3x3 shortcut on the per-wave DMA ring: parity, then a
# same-box A/B against the LDS-staged shortcut (SESA_CONV_SCR=0); HTDemucs fp16mix (fp16 attention + convs):
# parity and bench against bf16x3.
set -e
O=gpurun_out/r04f
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04f] $(date +%T) tokgemm_bench f16"
timeout -k 10 240 ./tools/tokgemm_bench 198648 f16 > $O/tokgemm_f16.txt 2>&1
echo "[r04f] $(date +%T) parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_htdemucs.py -v --timeout 300 \
  --timeout-method thread -k "levels or matrix or config0 or small_matches or full_segment" > $O/parity.txt 2>&1 || rc=$?
timeout -k 10 600 python -u -m pytest tests/test_scnet.py -v --timeout 300 --timeout-method thread \
  -k "small_matches or full_chunk_matches" > $O/parity_scnet.txt 2>&1 || rc=$?
if [ "${rc:-0}" != 0 ]; then echo "[r04f] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
run() {
  echo "[r04f] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py $3 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
run ring fp=1 "--steps 6 --warmup 1"
run lds SESA_CONV_SCR=0 "--steps 6 --warmup 1"
run ring_b fp=1 "--steps 6 --warmup 1"
run bsr_d2 SESA_TOKGEMM_DEPTH=2 "--model bs_roformer --steps 2 --warmup 1"
run bsr_d4 SESA_TOKGEMM_DEPTH=4 "--model bs_roformer --steps 2 --warmup 1"
run bsr_d3 SESA_TOKGEMM_DEPTH=3 "--model bs_roformer --steps 2 --warmup 1"
run htd_fp16mix fp=1 "--model htdemucs --precision fp16mix --steps 1 --warmup 1"
run htd_bf16x3 fp=1 "--model htdemucs --precision bf16x3 --steps 1 --warmup 1"
run htd_fp16mix_db SESA_HCONV_VARIANT=1 "--model htdemucs --precision fp16mix --steps 1 --warmup 1"
run scn_fp16mix fp=1 "--model scnet --precision fp16mix --steps 2 --warmup 1"
run scn_bf16x3 fp=1 "--model scnet --precision bf16x3 --steps 2 --warmup 1"
echo "[r04f] $(date +%T) done"
