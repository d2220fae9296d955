set -o pipefail
mkdir -p gpurun_out/r06
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06/prof_gap -o run -- python3 bench.py --model scnet --steps 1 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > gpurun_out/r06/gap_scnet.log 2>&1
python3 tools/gap_table.py gpurun_out/r06/prof_gap 20 0.5 | tee gpurun_out/r06/gap_scnet.txt
rm -rf gpurun_out/r06/prof_gap
