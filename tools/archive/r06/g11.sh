set -o pipefail
mkdir -p gpurun_out/r06
f() { local name=$1; shift; timeout -k 10 240 "$@" > gpurun_out/r06/$name.txt 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/r06/$name.txt | tail -1 | cut -c1-300; return $rc; }
for k in 0 1 2 3 4 5 6 7 8; do
  f vs11_form$k python -u tools/victim_stress.py form$k mfma 40 || exit 1
done
