#!/bin/bash
# Round artifacts on the product build: -m gpu tests, smoke(), bench lines (K3 default, K2,
# K5 short), rocprofv3 kernel-trace summary of the default bench, FETCH_SIZE / WRITE_SIZE
# PMC passes (separate runs) for the trace kernel, per-rank stripe timings.
set -o pipefail
TAG=${1:-final}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --config K2 --cpu-seconds 0 > $O/bench_k2.json 2>> $O/bench.err || exit 1
timeout -k 10 300 python bench.py --config K5 --steps 5 --warmup 2 --cpu-seconds 0 > $O/bench_k5.json 2>> $O/bench.err || exit 1
# profiled command: the default bench (whole 64-frame launches: 128 warmup + 512 timed) without
# the side measurements, so rocprofv3's per-launch average and the line's kernel_avg_us
# describe the same kind of launches
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench \
  -- python3 bench.py --cpu-seconds 0 --exhaustive-steps 0 --per-frame-steps 0 \
  > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
grep '^{' $O/prof.log > $O/bench_profiled.json; cat $O/bench_profiled.json
head -4 $O/prof/bench_kernel_stats.csv
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc -o culled_$c \
    -- python3 bench.py --cpu-seconds 0 --exhaustive-steps 0 --per-frame-steps 0 --steps 128 > $O/pmc_$c.log 2>&1 \
    || { echo "pmc $c failed"; tail -5 $O/pmc_$c.log; exit 1; }
done
FRAMES_PER_LAUNCH=64 python3 tools/pmc_summary.py $O/pmc_K3_culled.json trace_kernel $O/pmc/culled_FETCH_SIZE_counter_collection.csv $O/pmc/culled_WRITE_SIZE_counter_collection.csv | tail -8
timeout -k 10 300 python tools/rank_sim.py K3 50 > $O/rank_k3.jsonl 2>&1 || exit 1
cat $O/rank_k3.jsonl
timeout -k 10 300 python tools/rank_sim.py K5 10 > $O/rank_k5.jsonl 2>&1 || exit 1
grep '^{' $O/rank_k5.jsonl
