set -o pipefail
mkdir -p gpurun_out/r06
f() { local name=$1; shift; timeout -k 10 240 "$@" > gpurun_out/r06/$name.txt 2>&1; local rc=$?; tail -1 gpurun_out/r06/$name.txt | cut -c1-300; return $rc; }
f fs_none python -u tools/fft_stress.py none bf16x3 200 &&
f fs_mdx_x3 python -u tools/fft_stress.py mdx23c bf16x3 200 &&
f fs_mdx_x3_tdfold env SESA_TDF_VARIANT=old python -u tools/fft_stress.py mdx23c bf16x3 200 &&
f fs_bsr_x3 python -u tools/fft_stress.py bs_roformer bf16x3 200 &&
f fs_bsr_x3_noglds env SESA_TOKGEMM_GLDS=0 python -u tools/fft_stress.py bs_roformer bf16x3 200 &&
f fs_mdx_f16 python -u tools/fft_stress.py mdx23c fp16mix 200 &&
f st_mdx_x3_tdfold env SESA_TDF_VARIANT=old python -u tools/streams_trace.py mdx23c bf16x3 3 12 0 &&
f st_bsr_x3_noglds env SESA_TOKGEMM_GLDS=0 python -u tools/streams_trace.py bs_roformer bf16x3 3 6 0
