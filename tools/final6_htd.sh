#!/bin/bash
# HTDemucs evidence again after its bench default moved to two streams (bench.py DEFAULT_STREAMS): the configs[3] line,
# the owned rank-share line, the kernel trace.
set -e
O=gpurun_out/final6
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python bench.py --model htdemucs --steps 2 --warmup 1 --cpu-sample-chunks 8 > $O/bench_htdemucs_s2.json 2> $O/bench_htdemucs_s2.err
timeout -k 10 300 python bench.py --model htdemucs --rank-share 8 --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/bench_htdemucs_share8_s2.json 2> $O/bench_htdemucs_share8_s2.err
for n in htdemucs_s2 htdemucs_share8_s2; do
  python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['streams'], r['class'], r['frac'], r.get('traffic_over_algorithmic'), d.get('parity_rms'), (d.get('pcie_inclusive') or {}).get('value'), (d.get('cpu_baseline') or {}).get('value'))" $O/bench_$n.json $n
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_htd_s2 -o run -- python3 bench.py --model htdemucs --steps 1 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > $O/prof_htd_s2.json 2> $O/prof_htd_s2.err
python3 tools/rocprof_summary.py $O/prof_htd_s2 $O/kernel_stats_htdemucs_s2.txt > /dev/null
rm -rf $O/prof_htd_s2
