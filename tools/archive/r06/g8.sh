set -o pipefail
mkdir -p gpurun_out/r06
f() { local name=$1; shift; timeout -k 10 240 "$@" > gpurun_out/r06/$name.txt 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/r06/$name.txt | tail -2 | cut -c1-300; return $rc; }
for v in pk fma lds; do
  f vs_${v}_none python -u tools/victim_stress.py $v none 60 || exit 1
  f vs_${v}_mfma python -u tools/victim_stress.py $v mfma 60 || exit 1
done
