# g1dw L2-prefetch A/B (round 3): isolated medians (knob_ab), HBM fetch per launch
# (FETCH_SIZE), and the pipeline bench per variant, interleaved.  Measured: g1dw 6
# (prefetch of the next round's A rows) 362-364 us vs 383-391 without (4); a second
# load per line (both 64-B halves) 360 vs 362 (noise); also prefetching the round after
# next 371 us and 1.613-1.622M vs 1.628-1.645M ROIs/s in the pipeline, fetch 750 MB vs
# 410 MB per launch (2 x FETCH_SIZE).  Only 4 / 6 remain in the library.
set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
export TMPDIR=/tmp
timeout -k 10 180 python tools/exp/knob_ab.py g1dw "g1dw=6" "g1dw=4" > gpurun_out/g1pf.log 2>&1 || exit 1
for v in 4 6; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/g1pmc_$v -o run --output-format csv -- python3 tools/exp/g1_only.py $v > /dev/null 2>&1 || exit 1
done
for r in 1 2; do
  for v in 6 4; do
    TRK_TUNE=g1dw=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/g1pf_bench_${v}_$r.log 2>&1 || exit 1
    grep -o '"value": [0-9.]*' gpurun_out/g1pf_bench_${v}_$r.log | head -1 | sed "s/^/g1dw=$v r$r /"
  done
done
echo done
