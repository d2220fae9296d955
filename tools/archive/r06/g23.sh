set -o pipefail
mkdir -p gpurun_out/r06
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() { local name=$1; shift; env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/prof_g23_$name -o run -- python3 -u bench.py --model scnet --steps 1 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > gpurun_out/r06/g23_$name.log 2>&1 || return 1; python3 tools/rocprof_summary.py gpurun_out/r06/prof_g23_$name > gpurun_out/r06/g23_stats_$name.txt; rm -rf gpurun_out/r06/prof_g23_$name; echo "== $name"; grep -E "lstm|tok_gemm|gn_apply" gpurun_out/r06/g23_stats_$name.txt | cut -c1-150; }
run p2 SESA_SCN_P16=2 && run p0 SESA_SCN_P16=0
