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
# Round-5 steps, each mapped to the verdict item it serves (VERDICT.md "Next round: do this"):
#   tests / smoke            items 1, 3, 4: the GPU suite (weighted EP > 1 tolerance, masked full-size C3,
#                            local bypass, the cut library) and the driver's smoke
#   bench8gloo               item 2: the driver's N = 8 command, self-launched, 8 gloo ranks on one GPU
#   bench2gloo / bench4gloo  item 3: phases.exchange_ms with the local bypass in a rehearsal line
#   pmcstep                  item 3: PMC of the whole EP = 8 step (phase A + exchange + phase B) with and
#                            without the local bypass (tools/pmc_ep.py, summarize_prof.py step)
#   pmc / pmcfold / pmcep    item 6: same-build traffic for the final bench lines (N = 1 and N > 1)
#   benchjson / profdefault  item 6: one bench line of the final build and the driver's command under rocprofv3
for step in "$@"; do
    case $step in
        tests)  run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread ;;
        smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        fullweighted) # item 1: the full-size gating-weighted cases with their per-rank calc_diff printed
                run fullweighted 600 python -u -m pytest tests/test_fullsize_gpu.py -k gating_weighted -s -q --timeout 170 --timeout-method thread ;;
        bench)  run bench 600 python bench.py ;;
        benchjson) run bench 600 python bench.py && grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json ;;
        profdefault) # the driver's exact command under rocprofv3; per-loop averages from the kernel trace
                run rocprofdef 900 rocprofv3 --kernel-trace --stats -d $OUT/profdef -o prof --output-format csv -- python3 bench.py
                python tools/summarize_prof.py timed $OUT/profdef/prof_kernel_trace.csv "combine_rows_kernel<2," $OUT/profdef_timed.md "combine steps + kernel-alone loop (value; roofline.kernel_us),token-major layout reference (roofline.same_run_token_major_rows)" ;;
        bench2gloo) export DEEPEP_BENCH_BACKEND=gloo; run bench2gloo 600 python3 bench.py --gpus 2 --steps 10 --warmup 3; unset DEEPEP_BENCH_BACKEND ;;
        bench4gloo) export DEEPEP_BENCH_BACKEND=gloo; run bench4gloo 900 python3 bench.py --gpus 4 --steps 4 --warmup 2; unset DEEPEP_BENCH_BACKEND ;;
        bench8gloo) # the driver's N = 8 command form (bench.py starts 8 ranks + 8 xGMI preflight children), gloo
                # in place of RCCL since the 8 ranks share this one GPU; wall time in the line (launch.wall_s)
                export DEEPEP_BENCH_BACKEND=gloo; run bench8gloo 900 python3 bench.py --gpus 8 --steps 20 --warmup 5; unset DEEPEP_BENCH_BACKEND
                grep '^{' $OUT/bench8gloo.log | tail -1 > $OUT/bench8gloo.json || true ;;
        pmc)    for c in FETCH_SIZE WRITE_SIZE; do
                    run pmc_$c 300 timeout -s KILL 120 rocprofv3 --pmc $c -d $OUT/pmc_$c -o pmc --output-format csv -- python3 tools/pmc_run.py
                done ;;
        pmcfold) # fold this build's PMC passes (the `pmc` step) into profiles/pmc_traffic.json, so the bench
                 # line run after it in the same call carries measured traffic; the file comes back in $OUT
                run pmcfold 120 python tools/summarize_prof.py pmc profiles/pmc_traffic.json \
                    combine_fused_weighted_t8192_h7168_k8 1057488896 \
                    $(find $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE -name '*counter_collection.csv')
                cp profiles/pmc_traffic.json $OUT/pmc_traffic.json ;;
        pmcep)  # phase A of the EP = N combine (bench.py's inputs, ranks simulated on one GPU): PMC passes, folded
                # into profiles/pmc_traffic.json so an N > 1 bench line of this build carries measured traffic
                for n in 2 4 8; do
                    for c in FETCH_SIZE WRITE_SIZE; do
                        run pmcep${n}_$c 300 timeout -s KILL 240 rocprofv3 --pmc $c -d $OUT/pmcep${n}_$c -o pmc --output-format csv -- python3 tools/pmc_ep.py $n
                    done
                    run pmcepfold$n 120 python tools/summarize_prof.py ep profiles/pmc_traffic.json $OUT/pmc_ep${n}_meta.json \
                        $(find $OUT/pmcep${n}_FETCH_SIZE $OUT/pmcep${n}_WRITE_SIZE -name '*counter_collection.csv')
                    run pmcstepfold$n 120 python tools/summarize_prof.py step $OUT/pmc_step_ep${n}.json $OUT/pmc_ep${n}_meta.json \
                        $(find $OUT/pmcep${n}_FETCH_SIZE $OUT/pmcep${n}_WRITE_SIZE -name '*counter_collection.csv')
                    run pmcstepfold2$n 60 python tools/summarize_prof.py stepfold profiles/pmc_traffic.json $OUT/pmc_step_ep${n}.json
                done
                cp profiles/pmc_traffic.json $OUT/pmc_traffic.json ;;
        pmcstep) # the whole EP = N step with the diagonal travelling (DEEPEP_LOCAL_BYPASS=0), beside `pmcep`'s
                 # bypass passes: the difference is the own-rank rows' copy
                for n in 2 8; do
                    for c in FETCH_SIZE WRITE_SIZE; do
                        export DEEPEP_LOCAL_BYPASS=0
                        run pmcnb${n}_$c 300 timeout -s KILL 240 rocprofv3 --pmc $c -d $OUT/pmcnb${n}_$c -o pmc --output-format csv -- python3 tools/pmc_ep.py $n
                        unset DEEPEP_LOCAL_BYPASS
                    done
                    run pmcnbfold$n 120 python tools/summarize_prof.py step $OUT/pmc_step_ep${n}_nobypass.json $OUT/pmc_ep${n}_nobypass_meta.json \
                        $(find $OUT/pmcnb${n}_FETCH_SIZE $OUT/pmcnb${n}_WRITE_SIZE -name '*counter_collection.csv')
                done ;;
        cumask) run cumask 120 python tools/probe_cumask.py ;;
        kdisp)  run kdisp 300 python tools/kdispatch.py ;;
        khost)  run khost 300 python tools/khost.py ;;
        *) echo "unknown step $step" ;;
    esac
done
