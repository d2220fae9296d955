set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 900 python -u -m pytest tests/test_scnet.py tests/test_ensemble_models.py tests/test_ensemble.py -m gpu -x -q -rA --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/gputest_g18.txt 2>&1; rc=$?
grep -E "rms|passed|failed" gpurun_out/r06/gputest_g18.txt | tail -14
[ $rc -eq 0 ] || exit $rc
for m in scnet ensemble; do
  timeout -k 10 500 python -u bench.py --model $m --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06/g18_bench_$m.json 2> gpurun_out/r06/g18_bench_$m.log || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['parity']['worst_rms'], {k: v['ms_per_step'] for k, v in d['kernel_classes'].items()})" gpurun_out/r06/g18_bench_$m.json
done
