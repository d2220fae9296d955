#!/bin/bash
# SCNet --streams 1 vs 2 vs 3, same box
set -o pipefail
mkdir -p gpurun_out/r06
for s in 1 2 3 1; do
  timeout -k 10 400 python -u bench.py --model scnet --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-pcie --streams $s > gpurun_out/r06/scn_str_$s.json 2> gpurun_out/r06/scn_str_$s.log || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['config']['exec_batch'])" gpurun_out/r06/scn_str_$s.json
done
