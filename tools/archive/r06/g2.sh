set -o pipefail
mkdir -p gpurun_out/r06
run() { local name=$1; shift; timeout -k 10 300 python -u tools/streams_trace.py "$@" > gpurun_out/r06/$name.txt 2>&1; local rc=$?; tail -2 gpurun_out/r06/$name.txt | cut -c1-400; return $rc; }
run t2_mdx_x3 mdx23c bf16x3 3 12 1 &&
run t2_mdx_f16 mdx23c fp16mix 3 8 1 &&
run t2_bsr_f16 bs_roformer fp16 3 6 1 &&
run t2_bsr_x3 bs_roformer bf16x3 3 6 1
