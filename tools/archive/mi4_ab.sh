#!/bin/bash
# fp16 TFC convs on the 32-row dx-major tile (conv3x3_db_kernel<MI4>): GPU parity of the fp16 / MDX23C tests,
# then a same-box bench A/B against the 16-row tile (SESA_CONV_MI4=0), both with act_split fp16 planes.
set -e
O=gpurun_out/mi4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[mi4] $(date +%T) tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread \
  -k "fp16 or full_chunk or small or stress or config0" > $O/gputest.log 2>&1
run() {
  echo "[mi4] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
run mi4 fp=1
run mi2 SESA_CONV_MI4=0
run mi4b fp=1
run mi2b SESA_CONV_MI4=0
echo "[mi4] $(date +%T) done"
