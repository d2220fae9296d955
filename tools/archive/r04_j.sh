#!/bin/bash
# Round 4: BS-Roformer QKV epilogue -> one fp16 plane read by the fp16 attention (SESA_BSR_QKV16 A/B);
# HTDemucs fp16mix with fp16 transformer / channel Linears: parity and bench.
set -e
O=gpurun_out/r04j
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04j] $(date +%T) parity"
timeout -k 10 600 python -u -m pytest tests/test_bsr.py tests/test_htdemucs.py tests/test_amp_precision.py -v -s \
  --timeout 300 --timeout-method thread -k "fp16 or full_segment or small_matches or demucs_mode or amp" \
  > $O/parity.txt 2>&1 || rc=$?
if [ "${rc:-0}" != 0 ]; then echo "[r04j] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
run() {
  echo "[r04j] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py $3 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
run bsr_q16 fp=1 "--model bs_roformer --steps 2 --warmup 1"
run bsr_q32 SESA_BSR_QKV16=0 "--model bs_roformer --steps 2 --warmup 1"
run bsr_q16b fp=1 "--model bs_roformer --steps 2 --warmup 1"
run bsr_q32b SESA_BSR_QKV16=0 "--model bs_roformer --steps 2 --warmup 1"
run htd fp=1 "--model htdemucs --steps 1 --warmup 1"
run htd_b fp=1 "--model htdemucs --steps 1 --warmup 1"
echo "[r04j] $(date +%T) done"
