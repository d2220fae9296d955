#!/bin/bash
# MDX23C and BS-Roformer evidence again after their bench default moved to two streams (bench.py DEFAULT_STREAMS)
set -e
O=gpurun_out/final6
mkdir -p $O
line() {
  local n=$1 s=$2; shift 2
  timeout -k 10 $s python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err
  python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['streams'], d['config']['exec_batch'], r['class'], r['frac'], r.get('traffic_over_algorithmic'), d.get('parity_rms'), (d.get('pcie_inclusive') or {}).get('value'), (d.get('cpu_baseline') or {}).get('value'))" $O/bench_$n.json $n
}
line mdx23c_s2 500
line mdx23c_share8_s2 300 --rank-share 8 --no-cpu-baseline --no-parity
line bs_roformer_s2 600 --model bs_roformer --steps 3 --warmup 1 --cpu-sample-chunks 8
