#!/bin/bash
# Round 6: BS-Roformer cross-stream discrepancy vs the LDS wait before barriers (tools/barrier_scan.py).
# tools/streams_check.py (4-min track, demix_device streams 1 vs 2) on three builds of libsesa:
#   head: as committed before the fix; fft: only the FFT stage-loop barrier of fft1024 waits (sesa_sync);
#   all:  the built in-tree library (the round-6 A/B ran the blanket form, every __syncthreads as sesa_sync).
# Then the in-tree build's bench lines for BS-Roformer and MDX23C (the cost of the waits).
set -o pipefail
O=gpurun_out/sync_ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-head fft all}; do
  lib=""
  [ "$v" = all ] || lib="$GRAFT_REPO_ROOT/tools/_ab/libsesa_$v.so"
  echo "[sync_ab] $(date +%T) streams_check $v"
  if [ -n "$lib" ]; then export SESA_LIB=$lib; else unset SESA_LIB; fi
  timeout -k 10 400 python -u tools/streams_check.py bs_roformer fp16 4 > $O/sc_$v.txt 2>&1
  rc=$?; grep RESULT $O/sc_$v.txt; [ $rc -eq 0 ] || exit $rc
done
unset SESA_LIB
if [ -n "$BENCH" ]; then
  for m in bs_roformer mdx23c; do
    echo "[sync_ab] $(date +%T) bench $m"
    timeout -k 10 400 python -u bench.py --model $m --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$m.txt 2>&1
    rc=$?; tail -c 600 $O/bench_$m.txt; [ $rc -eq 0 ] || exit $rc
  done
fi
