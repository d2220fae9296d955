#!/bin/bash
# Round 5 lease E: the GPU suite on the tree (MDMA default, HTDemucs DConv apply / Gram / LDS-staged k3 conv, ensemble
# gate over three fixtures x seven methods), then benches: HTDemucs (A/B of the DConv kernels), BS-Roformer (A/B of the
# persistent staggered token GEMMs), ensemble (blend parity), MDX23C.
set -e
O=gpurun_out/r05e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05e] $(date +%T) gpu suite"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s > $O/gputest.txt 2>&1 || rc=$?
tail -3 $O/gputest.txt
if [ "${rc:-0}" != 0 ]; then echo "[r05e] gpu suite rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
b() {
  echo "[r05e] $(date +%T) bench $1"
  timeout -k 10 400 env $2 python bench.py $3 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
b htd "X=1" "--model htdemucs --steps 3 --warmup 1"
b htd_old "SESA_HTD_DCAPPLY=0 SESA_HTD_DCCONV=0" "--model htdemucs --steps 3 --warmup 1 --no-parity"
b bsr "X=1" "--model bs_roformer --steps 3 --warmup 1 --no-parity"
b bsr_pers1 "SESA_TOKGEMM_PERS=1 SESA_TOKGEMM_STAGGER=1" "--model bs_roformer --steps 3 --warmup 1"
b bsr_pers2 "SESA_TOKGEMM_PERS=1 SESA_TOKGEMM_STAGGER=2" "--model bs_roformer --steps 3 --warmup 1 --no-parity"
b bsr2 "X=1" "--model bs_roformer --steps 3 --warmup 1 --no-parity"
b ens "X=1" "--model ensemble --steps 3 --warmup 1"
b mdx "X=1" "--steps 5 --warmup 1"
echo "[r05e] $(date +%T) done"
