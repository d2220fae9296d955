#!/bin/bash
# Round 4: BS-Roformer band attention with heads looped per workgroup (SESA_ATTN_BAND_HPW A/B): parity (fp16 goldens,
# BS- and Mel-Band-Roformer) and same-box benches.
set -e
O=gpurun_out/r04s
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04s] $(date +%T) parity"
timeout -k 10 600 python -u -m pytest tests/test_bsr.py -v -s --timeout 300 --timeout-method thread -k "fp16" \
  > $O/parity.txt 2>&1 || rc=$?
if [ "${rc:-0}" != 0 ]; then echo "[r04s] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
run() {
  echo "[r04s] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py $3 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
run hpw4 fp=1 "--model bs_roformer --steps 2 --warmup 1"
run hpw1 SESA_ATTN_BAND_HPW=1 "--model bs_roformer --steps 2 --warmup 1"
run hpw8 SESA_ATTN_BAND_HPW=8 "--model bs_roformer --steps 2 --warmup 1"
run hpw2 SESA_ATTN_BAND_HPW=2 "--model bs_roformer --steps 2 --warmup 1"
run hpw4b fp=1 "--model bs_roformer --steps 2 --warmup 1"
echo "[r04s] $(date +%T) done"
