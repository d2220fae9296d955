#!/bin/bash
# Round 4: fp16 token GEMM half tile (256 x 128, two workgroups per CU) vs the 256 x 256 depth-3 ring:
# microbench (identity checked), BS-Roformer parity with the half tile, same-box A/B end to end.
set -e
O=gpurun_out/r04g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04g] $(date +%T) tokgemm_bench f16"
timeout -k 10 240 ./tools/tokgemm_bench 198648 f16 > $O/tokgemm_f16.txt 2>&1
echo "[r04g] $(date +%T) bsr parity (half tile)"
SESA_TOKGEMM_HT=1 timeout -k 10 600 python -u -m pytest tests/test_bsr.py -v -s --timeout 300 --timeout-method thread \
  -k "fp16" > $O/parity_bsr_ht.txt 2>&1 || rc=$?
if [ "${rc:-0}" != 0 ]; then echo "[r04g] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
run() {
  echo "[r04g] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py $3 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
run bsr_d3 fp=1 "--model bs_roformer --steps 2 --warmup 1"
run bsr_ht SESA_TOKGEMM_HT=1 "--model bs_roformer --steps 2 --warmup 1"
run bsr_d3b fp=1 "--model bs_roformer --steps 2 --warmup 1"
run bsr_htb SESA_TOKGEMM_HT=1 "--model bs_roformer --steps 2 --warmup 1"
echo "[r04g] $(date +%T) done"
