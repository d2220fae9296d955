set -o pipefail
mkdir -p gpurun_out/r06
f() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/r06/$name.txt 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/r06/$name.txt | grep -E "RESULT|Error|error" | tail -2 | cut -c1-300; return $rc; }
f g12_fs_mfma python -u tools/fft_stress.py agg:mfma x 200 &&
f g12_fs_mdx python -u tools/fft_stress.py mdx23c bf16x3 200 &&
f g12_st_mdx python -u tools/streams_trace.py mdx23c fp16mix 3 12 0 &&
f g12_st_mdx2 python -u tools/streams_trace.py mdx23c bf16x3 2 8 0 &&
f g12_st_bsr python -u tools/streams_trace.py bs_roformer fp16 3 8 0 &&
f g12_st_scn python -u tools/streams_trace.py scnet fp16mix 3 8 0 &&
f g12_st_htd python -u tools/streams_trace.py htdemucs fp16mix 3 8 0 &&
for m in mdx23c bs_roformer scnet htdemucs; do
  for lib in new old; do
    if [ $lib = old ]; then export SESA_LIB=$PWD/tools/_canary/libsesa_slp.so; else unset SESA_LIB; fi
    timeout -k 10 400 python -u bench.py --model $m --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > gpurun_out/r06/g12_bench_${m}_$lib.json 2> gpurun_out/r06/g12_bench_${m}_$lib.log || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" gpurun_out/r06/g12_bench_${m}_$lib.json
  done
done
