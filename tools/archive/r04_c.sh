#!/bin/bash
# Round 4: side-stream diagnostic; fp16mix with the fp16 decoder TDF Linears (parity on every full-width
# fixture + same-box A/B of the TDF plan); SCNet register-blocked ConvolutionModule head (parity + A/B);
# HTDemucs / SCNet --enable_amp deviations printed.
set -e
O=gpurun_out/r04c
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04c] $(date +%T) streams diagnostic"
timeout -k 10 120 python tools/streams_debug.py > $O/streams_debug.txt 2>&1
echo "[r04c] $(date +%T) parity"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_amp_precision.py tests/test_scnet.py -v -s \
  --timeout 300 --timeout-method thread -k "levels or amp or fp16mix or scnet or stress or config0" > $O/parity.txt 2>&1 || rc=$?
if [ "${rc:-0}" != 0 ]; then echo "[r04c] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
run() {
  echo "[r04c] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py $3 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
run mix_tdf16 fp=1 "--steps 10 --warmup 2"
run mix_tdf3 SESA_TDF_PLAN=3333333333333333 "--steps 10 --warmup 2"
run mix_tdf16b fp=1 "--steps 10 --warmup 2"
run scnet_rb fp=1 "--model scnet --steps 3 --warmup 1"
run scnet_old SESA_SCN_CM_RB=0 "--model scnet --steps 3 --warmup 1"
echo "[r04c] $(date +%T) done"
