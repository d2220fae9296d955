#!/bin/bash
# Round 5 lease F: token-GEMM epilogue without scratch spills + HTDemucs DConv variants: the BS-Roformer / HTDemucs /
# SCNet parity tests, then per-kernel rocprofv3 stats of HTDemucs in each DConv configuration and of BS-Roformer.
set -e
O=gpurun_out/r05f
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05f] $(date +%T) parity (bsr, htdemucs, scnet)"
timeout -k 10 900 python -u -m pytest tests/test_bsr.py tests/test_htdemucs.py tests/test_scnet.py -m gpu -v --timeout 300 \
  --timeout-method thread -s > $O/parity.txt 2>&1 || rc=$?
tail -2 $O/parity.txt
if [ "${rc:-0}" != 0 ]; then echo "[r05f] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
p() {
  echo "[r05f] $(date +%T) $1"
  timeout -k 10 400 env $2 rocprofv3 --kernel-trace --stats -d $O/prof_$1 -o run -- python3 bench.py $3 --no-cpu-baseline --no-parity \
    > $O/bench_$1.json 2> $O/bench_$1.err
}
p htd_new "X=1" "--model htdemucs --steps 2 --warmup 1"
p htd_old "SESA_HTD_DCAPPLY=0 SESA_HTD_DCCONV=0 SESA_HTD_DCGRAM=0" "--model htdemucs --steps 2 --warmup 1"
p htd_conv_old "SESA_HTD_DCCONV=0" "--model htdemucs --steps 2 --warmup 1"
p bsr "X=1" "--model bs_roformer --steps 2 --warmup 1"
echo "[r05f] $(date +%T) done"
