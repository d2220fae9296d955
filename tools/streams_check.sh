#!/bin/bash
# tools/streams_check.py per model (full-size 4-min track, demix_device at streams 1 / 2)
set -o pipefail
mkdir -p gpurun_out/r06
for spec in "htdemucs fp16mix 16" "scnet fp16mix 16"; do
  set -- $spec
  timeout -k 10 500 python -u tools/streams_check.py $1 $2 $3 > gpurun_out/r06/sc_$1_$2.txt 2>&1; rc=$?; grep RESULT gpurun_out/r06/sc_$1_$2.txt; [ $rc -eq 0 ] || exit $rc
done
