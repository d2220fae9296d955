#!/bin/bash
# Build the contraction-kernel micro-benchmark (diagnostic) into tools/conv_bench.
set -e
cd "$(dirname "$0")/.."
C=sesa-audio-separation_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -I include -I $C tools/conv_bench.hip \
  -o tools/conv_bench "$@"
