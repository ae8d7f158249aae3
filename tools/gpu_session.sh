#!/bin/bash
# One GPU session on the gpurun box: tests, smoke, bench, rocprof kernel trace.
# Each GPU step has its own time limit; a fault/abort/timeout (anything but exit 0/1) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
run() {   # run <name> <timeout> <cmd...>
    local name=$1 tmo=$2; shift 2
    echo "=== $name: $*" | tee -a $OUT/session.log
    timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a $OUT/session.log
    tail -5 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
    return 0
}
for step in "$@"; do
    case $step in
        tests)  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread ;;
        xgmistress) run xgmistress 300 python -u -m pytest tests/test_xgmi_gpu.py -k full_size -x -q --timeout 170 --timeout-method thread ;;
        smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench)  run bench 600 python bench.py ;;
        benchc4) run bench_c4 600 python bench.py --fp8-dispatch --no-cpu-baseline --no-loopback ;;
        benchc5) run bench_c5 600 python bench.py --tokens 16384 --skew 4 --no-cpu-baseline --no-loopback ;;
        benchplain) run bench_plain 600 python bench.py --plain --no-cpu-baseline --no-loopback ;;
        prof)   run rocprof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-loopback --no-flushed --no-layout-ref --steps 20 --warmup 5 ;;
        profdefault) # the driver's exact command under rocprofv3; per-loop averages from the kernel trace
                run rocprofdef 900 rocprofv3 --kernel-trace --stats -d $OUT/profdef -o prof --output-format csv -- python3 bench.py
                python tools/summarize_prof.py timed $OUT/profdef/prof_kernel_trace.csv "combine_rows_kernel<2," $OUT/profdef_timed.md "combine steps + kernel-alone loop (value; roofline.kernel_us),token-major layout reference (roofline.same_run_token_major_rows)" ;;
        kbench) run kbench 600 python tools/kbench.py ;;
        kuc)    run kuc 600 python tools/kbench_uc.py ;;
        pcopy)  [ -f tools/libprobe_copy.so ] || hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o tools/libprobe_copy.so tools/probe_copy.hip
                run pcopy 600 python tools/probe_copy.py ;;
        kbisect) run kbisect 600 python tools/kbisect.py ;;
        pcopydst) export PCOPY_BLOCKS=128 PCOPY_BLOCKED=9,9 PCOPY_VARIANTS=1,4,8,40,42,48,88,28,200,201,48; run pcopydst 600 python tools/probe_copy.py; unset PCOPY_BLOCKS PCOPY_BLOCKED PCOPY_VARIANTS ;;
        klayout) run klayout 300 python tools/klayout.py ;;
        kwin)   run kwin 300 python tools/kwin.py ;;
        klayoutruns) export KLAYOUT_RUNS=1; run klayoutruns 400 python tools/klayout.py; unset KLAYOUT_RUNS ;;
        kflush) run kflush 300 python tools/kflush.py ;;
        kphase) run kphase 300 python tools/kphase.py ;;
        profphase) run profphase 300 rocprofv3 --kernel-trace --stats -d $OUT/profphase -o prof --output-format csv -- python3 tools/kphase_prof.py ;;
        kcu)    run kcu 300 python tools/kcu.py ;;
        kdisp)  run kdisp 300 python tools/kdispatch.py ;;
        koverlap) run koverlap 300 python tools/koverlap.py ;;
        kdispprof) export KDISPATCH_CPROFILE=1; run kdispprof 300 python tools/kdispatch.py; unset KDISPATCH_CPROFILE ;;
        profdisp) run profdisp 300 rocprofv3 --kernel-trace -d $OUT/profdisp -o prof --output-format csv -- python3 tools/kdispatch.py ;;
        cumask) run cumask 120 python tools/probe_cumask.py ;;
        pmclist) run pmclist 120 rocprofv3 --list-avail ;;
        smi)    run smi 60 rocm-smi --showclocks --showpower --showtemp ;;
        bench4gloo) # the driver's plain command form: bench.py starts its own 4 ranks (sharing the one GPU over gloo)
                export DEEPEP_BENCH_BACKEND=gloo; run bench4gloo 900 python3 bench.py --gpus 4 --steps 4 --warmup 2; unset DEEPEP_BENCH_BACKEND ;;
        kphasea) run kphasea 300 python tools/kphase_a.py ;;
        khost)  run khost 300 python tools/khost.py ;;
        kshapes) run kshapes 400 python tools/kshapes.py ;;
        koutplace) run koutplace 300 python tools/koutplace.py ;;
        kphaseb) run kphaseb 300 python tools/kphase_b.py ;;
        tlb)    # six separate processes: the fused kernel back to back under the UTCL1 translation counters (is a
                # fast process one with fewer TLB misses?)
                for i in 1 2 3 4 5 6; do
                    run tlb$i 150 timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum GRBM_GUI_ACTIVE -d $OUT/tlb$i -o pmc --output-format csv -- python3 tools/pmc_run.py --b2b
                done ;;
        pmcpolicy) # phase A's store policies at EP = 4 under memory-side and L2 counters (one pass per counter set)
                i=0
                for cs in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
                    i=$((i+1))
                    run pmcpol_$i 200 timeout -s KILL 150 rocprofv3 --pmc $cs -d $OUT/pmcpol_$i -o pmc --output-format csv -- python3 tools/pmc_policy.py 4
                done
                run pmcpolfold 60 python tools/summarize_prof.py policy $OUT/pmc_policy.json $OUT/pmc_policy_meta.json \
                    $(find $OUT/pmcpol_1 $OUT/pmcpol_2 $OUT/pmcpol_3 $OUT/pmcpol_4 -name '*counter_collection.csv') ;;
        kprefetch) [ -f tools/libprobe_prefetch.so ] || hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o tools/libprobe_prefetch.so tools/probe_prefetch.hip
                run kprefetch 400 python tools/kprefetch.py ;;
        bench2gloo) export DEEPEP_BENCH_BACKEND=gloo; run bench2gloo 600 python3 bench.py --gpus 2 --steps 10 --warmup 3; unset DEEPEP_BENCH_BACKEND ;;
        pmc)    for c in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum; do
                    run pmc_$c 300 timeout -s KILL 120 rocprofv3 --pmc $c -d $OUT/pmc_$c -o pmc --output-format csv -- python3 tools/pmc_run.py
                done ;;
        pmcfold) # fold this build's PMC passes (the `pmc` step) into profiles/pmc_traffic.json, so the bench
                 # line run after it in the same call carries measured traffic; the file comes back in $OUT
                run pmcfold 120 python tools/summarize_prof.py pmc profiles/pmc_traffic.json \
                    combine_fused_weighted_t8192_h7168_k8 1057488896 \
                    $(find $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE $OUT/pmc_TCC_EA0_RDREQ_sum $OUT/pmc_TCC_EA0_WRREQ_sum -name '*counter_collection.csv')
                cp profiles/pmc_traffic.json $OUT/pmc_traffic.json ;;
        benchjson) run bench 600 python bench.py && grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json ;;
        pmcep)  # phase A of the EP = N combine (bench.py's inputs, ranks simulated on one GPU): PMC passes, folded
                # into profiles/pmc_traffic.json so an N > 1 bench line of this build carries measured traffic
                for n in 2 4 8; do
                    for c in FETCH_SIZE WRITE_SIZE; do
                        run pmcep${n}_$c 300 timeout -s KILL 240 rocprofv3 --pmc $c -d $OUT/pmcep${n}_$c -o pmc --output-format csv -- python3 tools/pmc_ep.py $n
                    done
                    run pmcepfold$n 120 python tools/summarize_prof.py ep profiles/pmc_traffic.json $OUT/pmc_ep${n}_meta.json \
                        $(find $OUT/pmcep${n}_FETCH_SIZE $OUT/pmcep${n}_WRITE_SIZE -name '*counter_collection.csv')
                done
                cp profiles/pmc_traffic.json $OUT/pmc_traffic.json ;;
        pmcphases) for c in FETCH_SIZE WRITE_SIZE; do
                    run pmcph_$c 300 timeout -s KILL 120 rocprofv3 --pmc $c -d $OUT/pmcph_$c -o pmc --output-format csv -- python3 tools/pmc_phases.py
                done ;;
        pmccal) # request-size calibration of every phase kernel (incl. the dispatch copy): 3 passes
                run pmccal_ws 300 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_EA0_WRREQ_sum -d $OUT/pmccal_ws -o pmc --output-format csv -- python3 tools/pmc_phases.py
                run pmccal_rq 300 timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $OUT/pmccal_rq -o pmc --output-format csv -- python3 tools/pmc_phases.py
                run pmccal_fs 300 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmccal_fs -o pmc --output-format csv -- python3 tools/pmc_phases.py ;;
        pmcplain) for c in FETCH_SIZE WRITE_SIZE; do
                    run pmcp_$c 300 timeout -s KILL 120 rocprofv3 --pmc $c -d $OUT/pmcp_$c -o pmc --output-format csv -- python3 tools/pmc_run.py --plain
                done ;;
        *) echo "unknown step $step" ;;
    esac
done
