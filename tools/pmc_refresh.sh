#!/bin/bash
# HBM traffic per launch of the dominant kernel classes, on THIS tree, for bench.py's roofline.traffic:
#   bash tools/pmc_refresh.sh MODEL "CLASS=SUBSTR[|SUBSTR..]" ...   (run on the GPU box; GIT_SHA from the caller)
# One bench step of the real workload (same exec batch as the timed run) under two separate rocprofv3 --pmc
# passes (FETCH_SIZE, then WRITE_SIZE: MI355X_MICROARCH.md HBM section; FETCH_SIZE doubled for gfx950 in
# tools/pmc_traffic.py), each under its own time limit; the summaries are stamped with the kernel sources'
# sha (bench.py KSRC + the model's own source) and written to gpurun_out/pmc_<class>_<model>.json.
set -e
M=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
# the precision the default bench line of this model runs in (bench.py default_precision), stamped into the
# summaries (bench.py reports traffic only for a run in the same mode)
P=$(python3 -c "import bench; print(bench.default_precision('$M'))")
# --streams 1: one step, every launch in it a libsesa profile record (with several streams bench.py adds a single-stream
# roofline pass, and the counters would see both passes against one pass of records)
B="python3 bench.py --model $M --steps 1 --warmup 0 --streams 1 --no-cpu-baseline --no-parity --no-pcie --precision $P"
O=gpurun_out
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_${M}_f -o run -- $B > $O/pmc_${M}_f.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_${M}_w -o run -- $B > $O/pmc_${M}_w.log 2>&1
for spec in "$@"; do
  K=${spec%%=*}; S=${spec#*=}
  # stamped with the precision that class's kernels ran in (bench.py class_precision)
  SESA_PMC_PRECISION=$(python3 -c "import bench; print(bench.class_precision('$K', '$P', '$M'))") SESA_PMC_MODEL=$M \
    python3 tools/pmc_traffic.py $O/pmc_${M}_f $O/pmc_${M}_w "$S" $O/pmc_${K}_${M}.json $K
done
