# A/B of the fused kernel with and without write bursts (needs tools/wip/fused_write_burst.patch applied):
# bench.py alternately with DEEPEP_COMBINE_BURST=0 / 1, two rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2 3 4; do
  for b in 0 1; do
    DEEPEP_COMBINE_BURST=$b timeout -k 10 200 python bench.py --no-cpu-baseline --no-loopback --steps 100 --warmup 10 > gpurun_out/ab_${b}_$i.log 2>&1 || exit $?
    echo "burst=$b run=$i $(grep '^{' gpurun_out/ab_${b}_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["kernel_us"], r["frac"])')" | tee -a gpurun_out/ab.log
  done
done
