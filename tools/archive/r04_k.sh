#!/bin/bash
# Round 4: HTDemucs fp16mix with fp16 Linears and the cheaper conv-gather addressing: parity and bench; SCNet
# (conv-mode token GEMM shares the staging) parity + bench.
set -e
O=gpurun_out/r04k
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04k] $(date +%T) parity"
timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py tests/test_scnet.py -v -s --timeout 300 \
  --timeout-method thread -k "full_segment or small_matches or demucs_mode or full_chunk_matches or wide" \
  > $O/parity.txt 2>&1 || rc=$?
if [ "${rc:-0}" != 0 ]; then echo "[r04k] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
run() {
  echo "[r04k] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py $3 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
run htd fp=1 "--model htdemucs --steps 1 --warmup 1"
run htd_b fp=1 "--model htdemucs --steps 1 --warmup 1"
run scn fp=1 "--model scnet --steps 2 --warmup 1"
echo "[r04k] $(date +%T) done"
