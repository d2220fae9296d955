set -o pipefail
mkdir -p gpurun_out/r06
f() { local name=$1; shift; timeout -k 10 240 "$@" > gpurun_out/r06/$name.txt 2>&1; local rc=$?; tail -4 gpurun_out/r06/$name.txt | cut -c1-400; return $rc; }
f fs4_matmul python -u tools/fft_stress.py matmul x 200 &&
f fs4_elem python -u tools/fft_stress.py elementwise x 200 &&
f fs4_stft python -u tools/fft_stress.py stft x 200 &&
f fs4_mdx python -u tools/fft_stress.py mdx23c bf16x3 200
