#!/bin/bash
# Round 4: fp16 attention with the lazy O / l rescale: parity (BS-Roformer, Mel-Band, HTDemucs, the ensemble at full
# width) and same-box A/B against the previous tree's line (BS-Roformer, HTDemucs).
set -e
O=gpurun_out/r04q
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04q] $(date +%T) parity"
timeout -k 10 900 python -u -m pytest tests/test_bsr.py tests/test_htdemucs.py tests/test_ensemble_models.py -v -s --timeout 300 \
  --timeout-method thread -k "fp16 or full_segment or small_matches or full_width" > $O/parity.txt 2>&1 || rc=$?
if [ "${rc:-0}" != 0 ]; then echo "[r04q] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
run() {
  echo "[r04q] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py $3 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
run bsr fp=1 "--model bs_roformer --steps 2 --warmup 1"
run bsr_b fp=1 "--model bs_roformer --steps 2 --warmup 1"
run htd fp=1 "--model htdemucs --steps 1 --warmup 1"
echo "[r04q] $(date +%T) done"
