set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && timeout -k 10 200 python tools/prof_scan.py > gpurun_out/prof_scan.json 2>gpurun_out/prof_scan.err; echo rc=$?; cat gpurun_out/prof_scan.json; tail -3 gpurun_out/prof_scan.err
