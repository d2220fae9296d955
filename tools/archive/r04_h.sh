#!/bin/bash
# Round 4: fp16 FF1 output staged through LDS and stored as full lines (microbench with identity check; parity;
# same-box BS-Roformer A/B: depth-3 full tile vs half tile); HTDemucs signal-major STFT / iSTFT grids (parity +
# bench).
set -e
O=gpurun_out/r04h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04h] $(date +%T) tokgemm_bench f16"
timeout -k 10 240 ./tools/tokgemm_bench 198648 f16 > $O/tokgemm_f16.txt 2>&1
echo "[r04h] $(date +%T) parity"
timeout -k 10 600 python -u -m pytest tests/test_bsr.py tests/test_htdemucs.py -v -s --timeout 300 \
  --timeout-method thread -k "fp16 or full_segment or small_matches or demucs_mode" > $O/parity.txt 2>&1 || rc=$?
if [ "${rc:-0}" != 0 ]; then echo "[r04h] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
run() {
  echo "[r04h] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py $3 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
run bsr fp=1 "--model bs_roformer --steps 2 --warmup 1"
run bsr_ht SESA_TOKGEMM_HT=1 "--model bs_roformer --steps 2 --warmup 1"
run bsr_b fp=1 "--model bs_roformer --steps 2 --warmup 1"
run bsr_htb SESA_TOKGEMM_HT=1 "--model bs_roformer --steps 2 --warmup 1"
run htd fp=1 "--model htdemucs --steps 1 --warmup 1"
echo "[r04h] $(date +%T) done"
