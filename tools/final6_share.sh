#!/bin/bash
# The two owned-form rank-share lines of tools/final6.sh (PART b) again, after bench.py stopped applying the 1-GPU PMC
# traffic to a rank's share.
set -e
O=gpurun_out/final6
mkdir -p $O
timeout -k 10 300 python bench.py --rank-share 8 --no-cpu-baseline --no-parity > $O/bench_mdx23c_share8.json 2> $O/bench_mdx23c_share8.err
timeout -k 10 300 python bench.py --model htdemucs --rank-share 8 --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/bench_htdemucs_share8.json 2> $O/bench_htdemucs_share8.err
for n in mdx23c_share8 htdemucs_share8; do
  python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d['roofline']
print(sys.argv[2], d['value'], d['pcie_inclusive']['value'], r['class'], r['frac'], r.get('traffic'), r.get('traffic_source'))" $O/bench_$n.json $n
done
