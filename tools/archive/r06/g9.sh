set -o pipefail
mkdir -p gpurun_out/r06
f() { local name=$1; shift; timeout -k 10 240 "$@" > gpurun_out/r06/$name.txt 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/r06/$name.txt | tail -2 | cut -c1-300; return $rc; }
f vs_pkmix_mfma python -u tools/victim_stress.py pkmix mfma 60 &&
f fs9_noslp_mfma env FFT_VICTIM_LIB=tools/_canary/libspec_noslp.so python -u tools/fft_stress.py agg:mfma x 200 &&
f fs9_noslp_mdx env FFT_VICTIM_LIB=tools/_canary/libspec_noslp.so python -u tools/fft_stress.py mdx23c bf16x3 200 &&
f fs9_base_mfma python -u tools/fft_stress.py agg:mfma x 200
