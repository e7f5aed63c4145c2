# round-2 measurements: full -m gpu suite, smoke, default bench, decode kernel
# traces (C2 / C3 / dense 64 B) and the k_scan SQ counters on C3
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_r02_tests.sh || exit 1
bash tools/gpu_kt_decode.sh || exit 1
bash tools/gpu_pmc_scan.sh || exit 1
echo measured
