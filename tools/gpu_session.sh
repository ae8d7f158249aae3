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
# Round-6 steps, each mapped to the verdict item it serves (VERDICT.md "Next round: do this"):
#   ldsdma / ldsdmaprof      item 1: the LDS-DMA load-path experiment (timing, rocprof, PMC, both layouts); removed
#                            with the variant after the negative (results: profiles/r06a_ldsdma*, CHANGELOG round 6)
#   bench2def / bench8def    item 2: the driver's default N > 1 command on this one GPU: the RCCL preflight fails
#                            (duplicate GPU), the ranks agree, the headline falls back to xGMI, the line is complete
#   barrier                  item 3: the barrier tests' device-clock ordering evidence
#   pmcep (+ stepfold)       item 5: same-build step PMC per transport -> phases.hbm_bytes_per_rank
#   bench8gloo               item 5: the N = 8 gloo rehearsal line carrying phases.hbm_bytes_per_rank
#   tests / smoke / pmc / pmcfold / benchjson / profdefault
#                            item 6: the final build's suite, smoke, bench line, same-build PMC and rocprof
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
        barrier) run barrier 300 python -u -m pytest tests/test_barrier_gpu.py -x -v --timeout 150 --timeout-method thread ;;
        bench2def) run bench2def 420 python3 bench.py --gpus 2 --steps 10 --warmup 3
                grep '^{' $OUT/bench2def.log | tail -1 > $OUT/bench2def.json || true ;;
        bench8def) run bench8def 700 python3 bench.py --gpus 8 --steps 20 --warmup 5
                grep '^{' $OUT/bench8def.log | tail -1 > $OUT/bench8def.json || true ;;
        cumask) run cumask 120 python tools/probe_cumask.py ;;
        kdisp)  run kdisp 300 python tools/kdispatch.py ;;
        khost)  run khost 300 python tools/khost.py ;;
        *) echo "unknown step $step" ;;
    esac
done
