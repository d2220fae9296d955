set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_scnet.py -m gpu -x -q -rA --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/gputest_g17.txt 2>&1; rc=$?
grep -E "rms|passed|failed" gpurun_out/r06/gputest_g17.txt | tail -12
[ $rc -eq 0 ] || exit $rc
for ps in 3 2 1; do
  export SESA_SCN_LSTM_PASSES=$ps
  timeout -k 10 400 python -u bench.py --model scnet --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/r06/g17_bench_scnet_ps$ps.json 2> gpurun_out/r06/g17_bench_scnet_ps$ps.log || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['parity']['worst_rms'], d['kernel_classes']['lstm']['ms_per_step'], d['kernel_classes'].get('istft'))" gpurun_out/r06/g17_bench_scnet_ps$ps.json
done
