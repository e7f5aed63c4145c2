#!/bin/bash
# tools/gpu_round.sh -- the GPU passes of a round, one MI355X (run through gpurun:
#   gpurun --timeout N -- 'bash tools/gpu_round.sh STEP [STEP ...]').
# Every GPU step runs under its own time limit; the first failing step ends the
# script (no retries). Outputs go under gpurun_out/$ROUND/ (copy what is judged
# into profiles/$ROUND/).
#   tests        pytest -m gpu (whole suite, one process)
#   smoke        __graft_entry__.smoke()
#   bench        python bench.py (default: headline + extras + C1 + CPU baseline)
#   bench_quick  python bench.py --no-extra --no-cpu
#   share2       bench.py --gpus 2 --share-device (two ranks on device 0, gloo): the N-rank path on HIP
#   pmc          FETCH_SIZE / WRITE_SIZE passes of the headline kernel (separate runs)
#   pmc_rq       the TCC_EA0_RDREQ 32/64/128-B request counts of the headline kernel (sized reads)
#   prof_main    rocprofv3 kernel trace + stats of the headline bench
#   prof_decode  rocprofv3 kernel trace + stats of the C2/C3/dense/C5 stream decodes
#   prof_extra   rocprofv3 kernel trace + stats of C4 gather, TX encode, C5 descriptor mode
#   pmc_decode   FETCH_SIZE / WRITE_SIZE passes of the C3 decode (tools/run_decode.py c3)
#   pmc_extra    FETCH_SIZE / WRITE_SIZE passes of C4 (tools/run_c4.py) and TX (tools/run_tx.py)
#   sq_decode    SQ counters of the C3 decode kernels
#   trace        phase clocks of k_scan and per-workgroup timelines of the resolve kernels
#                (FWS_SCAN_PROF build: make -C flashws_amd/csrc prof, built beforehand)
set -o pipefail
ROUND=${ROUND:-r06}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$ROUND
mkdir -p "$O"
cd "$R" || exit 1
fail() { echo "step $1 failed (rc $2)"; tail -30 "$3"; exit 1; }
prof() {   # prof NAME TIMEOUT ARGS... : rocprofv3 with the program right after --
    local name=$1 t=$2; shift 2
    (cd /tmp && TMPDIR=/tmp timeout -k 10 "$t" rocprofv3 "$@") > "$O/$name.log" 2>&1 || fail "$name" $? "$O/$name.log"
}
for step in "$@"; do
    echo "== $step $(date +%T)"
    case $step in
    tests)
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
            > "$O/gpu_tests.log" 2>&1 || fail tests $? "$O/gpu_tests.log"
        tail -1 "$O/gpu_tests.log" ;;
    smoke)
        timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
            || fail smoke $? "$O/smoke.log"
        tail -1 "$O/smoke.log" ;;
    bench)
        timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err" || fail bench $? "$O/bench.err"
        cut -c1-600 "$O/bench.json" ;;
    bench_quick)
        timeout -k 10 300 python bench.py --no-extra --no-cpu > "$O/bench_quick.json" 2> "$O/bench_quick.err" \
            || fail bench_quick $? "$O/bench_quick.err"
        cut -c1-600 "$O/bench_quick.json" ;;
    share2)
        timeout -k 10 600 python bench.py --gpus 2 --share-device --no-cpu --steps 20 --warmup 5 \
            > "$O/share2.json" 2> "$O/share2.err" || fail share2 $? "$O/share2.err"
        cut -c1-2000 "$O/share2.json" ;;
    pmc)
        prof pmc_fetch 120 --pmc FETCH_SIZE -f csv -d "$O/pmc_fetch" -o run -- python3 "$R/bench.py" --no-extra --no-cpu --no-batch-extra --steps 10 --warmup 2
        prof pmc_write 120 --pmc WRITE_SIZE -f csv -d "$O/pmc_write" -o run -- python3 "$R/bench.py" --no-extra --no-cpu --no-batch-extra --steps 10 --warmup 2 ;;
    pmc_rq)      # sized read requests of the headline kernel (tools/pmc_summary.py --rdreq)
        prof pmc_rq 120 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -f csv -d "$O/pmc_rq" -o run -- python3 "$R/bench.py" --no-extra --no-cpu --no-batch-extra --steps 10 --warmup 2 ;;
    prof_main)
        prof prof_main 300 --kernel-trace --stats -f csv -d "$O/prof_main" -o run -- python3 "$R/bench.py" --no-extra --no-cpu ;;
    prof_decode)
        for c in c2 c3 dense c5_256m; do
            prof "prof_$c" 300 --kernel-trace --stats -f csv -d "$O/prof_$c" -o run -- python3 "$R/tools/run_decode.py" $c
        done ;;
    prof_extra)
        prof prof_c4 200 --kernel-trace --stats -f csv -d "$O/prof_c4" -o run -- python3 "$R/tools/run_c4.py"
        prof prof_tx 200 --kernel-trace --stats -f csv -d "$O/prof_tx" -o run -- python3 "$R/tools/run_tx.py"
        prof prof_c5d 300 --kernel-trace --stats -f csv -d "$O/prof_c5d" -o run -- python3 "$R/tools/run_c5_desc.py" ;;
    pmc_decode)
        prof pmc_dec_fetch 120 --pmc FETCH_SIZE -f csv -d "$O/pmc_dec_fetch" -o run -- python3 "$R/tools/run_decode.py" c3
        prof pmc_dec_write 120 --pmc WRITE_SIZE -f csv -d "$O/pmc_dec_write" -o run -- python3 "$R/tools/run_decode.py" c3 ;;
    pmc_extra)
        for c in c4 tx; do
            prof "pmc_${c}_fetch" 150 --pmc FETCH_SIZE -f csv -d "$O/pmc_${c}_fetch" -o run -- python3 "$R/tools/run_$c.py"
            prof "pmc_${c}_write" 150 --pmc WRITE_SIZE -f csv -d "$O/pmc_${c}_write" -o run -- python3 "$R/tools/run_$c.py"
        done ;;
    sq_decode)
        prof sq_dec 120 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM -f csv -d "$O/sq_dec" -o run -- python3 "$R/tools/run_decode.py" c3 ;;
    trace)
        timeout -k 10 300 python tools/prof_scan.py > "$O/prof_scan.json" 2> "$O/prof_scan.err" || fail trace $? "$O/prof_scan.err"
        timeout -k 10 300 python tools/prof_merge_trace.py > "$O/prof_merge_trace.json" 2> "$O/prof_merge_trace.err" \
            || fail trace $? "$O/prof_merge_trace.err" ;;
    dectests)
        timeout -k 10 900 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_configs.py -x -v --timeout 120 --timeout-method thread \
            > "$O/dec_tests.log" 2>&1 || fail dectests $? "$O/dec_tests.log"
        tail -1 "$O/dec_tests.log" ;;
    dropin)
        timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py -x -v --timeout 120 --timeout-method thread \
            > "$O/dropin_tests.log" 2>&1 || fail dropin $? "$O/dropin_tests.log"
        tail -1 "$O/dropin_tests.log" ;;
    tdec)
        timeout -k 10 300 python tools/time_decode.py 20 > "$O/time_decode.json" 2> "$O/time_decode.err" \
            || fail tdec $? "$O/time_decode.err"
        cat "$O/time_decode.err" | grep -v amdgpu.ids ;;
    kdec)
        for c in c3 dense; do
            prof "kdec_$c" 300 --kernel-trace --stats -f csv -d "$O/kdec_$c" -o run -- python3 "$R/tools/run_decode.py" $c 20
        done
        for c in c3 dense; do cut -d, -f1-5 "$O/kdec_$c/run_kernel_stats.csv" | head -12; done ;;
    utf8tests)
        timeout -k 10 600 python -u -m pytest tests/test_gpu_sorted_utf8.py tests/test_gpu_decode.py tests/test_gpu_configs.py -k "utf8 or c5 or C5 or text" -x -v --timeout 120 --timeout-method thread \
            > "$O/utf8_tests.log" 2>&1 || fail utf8tests $? "$O/utf8_tests.log"
        tail -1 "$O/utf8_tests.log" ;;
    ab_c5)       # A/B: UTF-8 check forms (FWS_LIB_VARIANT=swar: make exp EXP_TAG=swar EXP_DEFS=-DFWS_UTF8_SWAR=1)
        for v in swar "" swar ""; do
            FWS_LIB_VARIANT=$v timeout -k 10 300 python bench.py --only c5d,c5s --no-cpu --no-batch-extra --steps 20 --warmup 5 \
                >> "$O/ab_c5.jsonl" 2>> "$O/ab_c5.err" || fail ab_c5 $? "$O/ab_c5.err"
            python3 -c "import json,sys;d=json.loads(open('$O/ab_c5.jsonl').read().splitlines()[-1]);e=d['extra'];print('variant=${v:-product}', e['C5_utf8_descriptor']['ms_per_step'], e['C5_utf8_text_decode']['ms_per_step'])"
        done ;;
    prof_extras)  # warm kernel stats per config: bench.py --only CFG under rocprofv3, stats of the timed window
        mkdir -p "$O/profiles"
        for c in ${PROF_CFGS:-c3 dense c2s c4 tx c5d c5s}; do
            prof "prof_$c" 400 --kernel-trace --stats -f csv -d "$O/prof_$c" -o run -- python3 "$R/bench.py" --only $c --no-cpu --no-batch-extra --no-pipelined --steps 20 --warmup 5
            grep '^{"metric"' "$O/prof_$c.log" | tail -1 > "$O/profiles/${c}_bench_line.json"
            last=20; case $c in c5*) last=16 ;; esac
            python3 tools/prof_window.py "$O/prof_$c/run_kernel_trace.csv" --last $last --out "$O/profiles/${c}_kernel_stats.csv" \
                --json "$O/profiles/${c}_window.json" --bench "$O/profiles/${c}_bench_line.json" > /dev/null || fail "window_$c" 1 "$O/prof_$c.log"
            cp "$O/prof_$c/run_kernel_stats.csv" "$O/profiles/${c}_kernel_stats_all.csv"
            python3 -c "import json;d=json.load(open('$O/profiles/${c}_window.json'));k=sorted(d['kernels'].items(),key=lambda x:-x[1]['window_avg_us'])[:3];print('$c',d.get('bench_ms_per_step'),[(n[:40],v['window_avg_us']) for n,v in k])"
        done ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
echo "all steps done $(date +%T)"
