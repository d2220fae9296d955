set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py tests/test_scnet.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/gputest_g21.txt 2>&1; rc=$?
tail -2 gpurun_out/r06/gputest_g21.txt
[ $rc -eq 0 ] || exit $rc
for lib in new base new2 base2; do
  if [ ${lib%2} = base ]; then export SESA_LIB=$PWD/tools/_canary/libsesa_r06base.so; else unset SESA_LIB; fi
  timeout -k 10 400 python -u bench.py --model htdemucs --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > gpurun_out/r06/g21_bench_htd_$lib.json 2> gpurun_out/r06/g21_bench_htd_$lib.log || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['kernel_classes']['istft'], d['kernel_classes']['stft'])" gpurun_out/r06/g21_bench_htd_$lib.json
done
unset SESA_LIB
timeout -k 10 400 python -u bench.py --model scnet --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/r06/g21_bench_scnet.json 2> gpurun_out/r06/g21_bench_scnet.log || exit 1
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['parity']['worst_rms'], {k: v['ms_per_step'] for k, v in d['kernel_classes'].items()})" gpurun_out/r06/g21_bench_scnet.json
