#!/bin/bash
# Round 4: MDX23C parity on the level / seed fixtures (every precision), the --enable_amp gate per model, the
# full-width ensemble, side streams; then a same-box A/B of the fp16mix plans against fp16 / fp16w2
# (configs[1] headline bench, no CPU leg).
set -e
O=gpurun_out/r04ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04ab] $(date +%T) conv_bench f16 (shortcut phase: LDS vs register-direct)"
timeout -k 10 300 ./tools/conv_bench 57 f16 > $O/conv_f16.txt 2>&1
echo "[r04ab] $(date +%T) parity"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_amp_precision.py tests/test_ensemble_models.py \
  -v --timeout 300 --timeout-method thread \
  tests/test_bsr.py -k "levels or matrix or amp or full_width or side_streams or fp16" > $O/parity.txt 2>&1 || rc=$?
# plain test failures (exit 1) still allow the bench; a crash, abort or time limit ends the script here
if [ "${rc:-0}" != 0 ]; then echo "[r04ab] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
run() {
  echo "[r04ab] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py --precision $3 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
run fp16 fp=1 fp16
run mix1311 SESA_F16_PLAN=1311111111111111 fp16mix
run mix1211 SESA_F16_PLAN=1211111111111111 fp16mix
run mix1321 SESA_F16_PLAN=1321111111111111 fp16mix
run fp16w2 fp=1 fp16w2
run fp16b fp=1 fp16
run mix1311b SESA_F16_PLAN=1311111111111111 fp16mix
echo "[r04ab] $(date +%T) done"
