set -o pipefail
mkdir -p gpurun_out/r06
t() { local name=$1; shift; env "$@" timeout -k 10 300 python -u -m pytest tests/test_ensemble_models.py -m gpu -q -rA -k "full_width and bench" --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/g19_$name.txt 2>&1; local rc=$?; echo "== $name"; grep -E "scnet stem|max_fft" gpurun_out/r06/g19_$name.txt; return $rc; }
t base A=1 && t band SESA_SCN_BAND_VALU=1 && t cm SESA_SCN_CM_VALU=1 && t lstm3 SESA_SCN_LSTM_PASSES=3 && t all3 SESA_SCN_BAND_VALU=1 SESA_SCN_CM_VALU=1 SESA_SCN_LSTM_PASSES=3
