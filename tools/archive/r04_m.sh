#!/bin/bash
# Round 4: MDX23C fp16 transposed up-convs (SESA_MDX_UP16 A/B) with the encoder-L0 fp16 TDF default: parity on
# every fixture, configs[0], same-box A/B; per-kernel HBM counters of one HTDemucs step (diagnostic for its
# fp32 VALU kernels).
set -e
O=gpurun_out/r04m
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04m] $(date +%T) parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_amp_precision.py -v -s --timeout 300 \
  --timeout-method thread -k "(levels and fp16mix) or config0 or full_size or matrix or (amp and mdx23c)" \
  > $O/parity.txt 2>&1 || rc=$?
if [ "${rc:-0}" != 0 ]; then echo "[r04m] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
run() {
  echo "[r04m] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py $3 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
run up16 fp=1 "--steps 6 --warmup 1"
run up3 SESA_MDX_UP16=0 "--steps 6 --warmup 1"
run up16b fp=1 "--steps 6 --warmup 1"
run up3b SESA_MDX_UP16=0 "--steps 6 --warmup 1"
echo "[r04m] $(date +%T) htdemucs per-kernel counters"
B="python3 bench.py --model htdemucs --steps 1 --warmup 0 --track-seconds 600 --no-cpu-baseline --no-parity"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_htd_f -o run -- $B > $O/pmc_htd_f.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_htd_w -o run -- $B > $O/pmc_htd_w.log 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_htd -o run -- $B > $O/prof_htd.log 2>&1
python3 tools/pmc_sq.py $O/pmc_htd_f $O/pmc_htd_w > $O/pmc_htd_kernels.txt 2>&1 || true
python3 tools/rocprof_summary.py $O/prof_htd $O/kernel_stats_htd600.txt > /dev/null || true
rm -rf $O/pmc_htd_f $O/pmc_htd_w $O/prof_htd
echo "[r04m] $(date +%T) done"
