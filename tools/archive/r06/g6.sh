set -o pipefail
mkdir -p gpurun_out/r06
f() { local name=$1; shift; timeout -k 10 240 "$@" > gpurun_out/r06/$name.txt 2>&1; local rc=$?; head -30 gpurun_out/r06/$name.txt | grep -v amdgpu.ids | cut -c1-300; return $rc; }
f cn2_all python -u tools/lds_canary.py mdx23c bf16x3 16384 20 256 8000 &&
f cn2_all8k python -u tools/lds_canary.py mdx23c bf16x3 8192 20 512 8000 &&
f cn2_down env SESA_DEBUG_ONLY=2 python -u tools/lds_canary.py mdx23c bf16x3 16384 20 256 8000 &&
f cn2_conv1 env SESA_DEBUG_ONLY=1 python -u tools/lds_canary.py mdx23c bf16x3 16384 20 256 8000
