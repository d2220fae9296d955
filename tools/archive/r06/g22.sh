set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_scnet.py -m gpu -x -q -rA --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/gputest_g22.txt 2>&1; rc=$?
grep -E "fp16mix rms|passed|failed" gpurun_out/r06/gputest_g22.txt | tail -4
[ $rc -eq 0 ] || exit $rc
for p in 2 0; do
  export SESA_SCN_P16=$p
  timeout -k 10 400 python -u bench.py --model scnet --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/r06/g22_bench_scnet_p$p.json 2> gpurun_out/r06/g22_bench_scnet_p$p.log || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['parity']['worst_rms'], {k: v['ms_per_step'] for k, v in d['kernel_classes'].items()})" gpurun_out/r06/g22_bench_scnet_p$p.json
done
