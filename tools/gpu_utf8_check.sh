# UTF-8 parity tests, then the C5 descriptor timing of the product library
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sorted_utf8.py tests/test_gpu_unmask.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/utf8_tests.log 2>&1 || { tail -30 gpurun_out/utf8_tests.log; exit 1; }
tail -1 gpurun_out/utf8_tests.log
bash tools/gpu_utf8_exp.sh "$@"
