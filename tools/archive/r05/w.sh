#!/bin/bash
# Round 5 lease W: the fp16 TDF Linears on deep LDS-DMA rings (tdf_dma_kernel<DEEP>, SESA_TDF_DEEP=1) -- MDX23C GPU
# parity tests with it, same-box configs[1] bench A / B (parity fixtures) / A2, kernel traces of A and B.
set -e
O=gpurun_out/r05w
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { echo "[r05w] $(date +%T) $*"; }
step tests deep
SESA_TDF_DEEP=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py > $O/tests_deep.txt 2>&1 || { tail -30 $O/tests_deep.txt; exit 1; }
tail -2 $O/tests_deep.txt
step bench A
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity > $O/bench_a.json 2> $O/bench_a.err
step bench B deep
SESA_TDF_DEEP=1 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_deep.json 2> $O/bench_deep.err
step bench A2
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity > $O/bench_a2.json 2> $O/bench_a2.err
step rocprof A
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pa -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $O/pa.json 2> $O/pa.err
python3 tools/rocprof_summary.py $O/pa $O/kernel_stats_a.txt > /dev/null
rm -rf $O/pa
step rocprof B
SESA_TDF_DEEP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pb -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $O/pb.json 2> $O/pb.err
python3 tools/rocprof_summary.py $O/pb $O/kernel_stats_deep.txt > /dev/null
rm -rf $O/pb
grep tdf_dma $O/kernel_stats_a.txt $O/kernel_stats_deep.txt || true
step done
