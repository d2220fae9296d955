#!/bin/bash
# Round 5 lease T: HTDemucs final evidence on the tree with the fused iSTFT default -- GPU tests, sha-stamped PMC
# traffic (hconv / simt / attn), the configs[3] bench line (CPU baseline, parity), rank-share 8, kernel-trace summary.
set -e
O=gpurun_out/r05t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { echo "[r05t] $(date +%T) $*"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/tests.txt 2>&1
step pmc
timeout -k 10 700 bash tools/pmc_refresh.sh htdemucs \
  "hconv=2, false, true, false|1, false, true, false|htd_rw3|htd_ctr" \
  "simt=htd_dc_|htd_item_stats|htd_gn_apply|htd_norm_freq|htd_norm_time" \
  "attn=attn_kernel|attn_f16_kernel" > $O/pmc_htdemucs.log 2>&1
rm -rf gpurun_out/pmc_*_f gpurun_out/pmc_*_w
cp gpurun_out/pmc_*_htdemucs.json profiles/
step bench
timeout -k 10 600 python bench.py --model htdemucs --steps 2 --warmup 1 --cpu-sample-chunks 8 > $O/bench_htdemucs.json 2> $O/bench_htdemucs.err
step share8
timeout -k 10 300 python bench.py --model htdemucs --rank-share 8 --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/bench_htdemucs_share8.json 2> $O/bench_htdemucs_share8.err
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_htdemucs -o run -- python3 bench.py --model htdemucs --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $O/prof_htdemucs.json 2> $O/prof_htdemucs.err
python3 tools/rocprof_summary.py $O/prof_htdemucs $O/kernel_stats_htdemucs.txt > /dev/null
rm -rf $O/prof_htdemucs
step done
