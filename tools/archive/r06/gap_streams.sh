#!/bin/bash
# Idle gaps of the MDX23C / HTDemucs / BS-Roformer steps (kernel trace), then the bench lines at --streams 1 vs 2
set -o pipefail
mkdir -p gpurun_out/r06
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for m in mdx23c htdemucs bs_roformer; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06/prof_gap_$m -o run -- python3 bench.py --model $m --steps 1 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > gpurun_out/r06/gap_$m.log 2>&1 || exit 1
  echo "== $m"; python3 tools/gap_table.py gpurun_out/r06/prof_gap_$m 6 0.5 | tee gpurun_out/r06/gap_$m.txt
  rm -rf gpurun_out/r06/prof_gap_$m
done
for m in mdx23c htdemucs bs_roformer; do
  for s in 1 2; do
    timeout -k 10 400 python -u bench.py --model $m --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-pcie --streams $s > gpurun_out/r06/str_${m}_$s.json 2> gpurun_out/r06/str_${m}_$s.log || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" gpurun_out/r06/str_${m}_$s.json
  done
done
