set -o pipefail
mkdir -p gpurun_out/r06
run() { local name=$1; shift; timeout -k 10 300 python -u tools/streams_trace.py "$@" > gpurun_out/r06/$name.txt 2>&1; local rc=$?; tail -3 gpurun_out/r06/$name.txt; return $rc; }
run st_mdx_x3_trace mdx23c bf16x3 3 12 1 &&
run st_mdx_x3_notrace mdx23c bf16x3 3 12 0 &&
run st_mdx_f16_trace mdx23c fp16mix 3 8 1 &&
run st_bsr_notrace bs_roformer fp16 3 6 0 &&
run st_scn_notrace scnet fp16mix 3 6 0 &&
run st_htd_notrace htdemucs fp16mix 3 6 0
