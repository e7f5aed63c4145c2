set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --no-extra --no-cpu --steps 10 --warmup 2 > $R/gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --no-extra --no-cpu --steps 10 --warmup 2 > $R/gpurun_out/pmc_write.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_main -o run -- python3 $R/bench.py --no-extra --no-cpu > $R/gpurun_out/prof_main.log 2>&1
echo done
