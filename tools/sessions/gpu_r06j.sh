#!/bin/bash
# Round 6: the driver's K3 command on the launch-timing tree (three times), the K2 / K4 / K5
# main lines, the default length, and the driver's command under rocprofv3 --kernel-trace
# --stats with the timed region's host stamps (RT_TIMELINE=1): the timed kernel's duration
# inside the region (tools/rocpd_stats.py RT_WINDOW) next to the line's kernel_avg_us.
set -o pipefail
TAG=${1:-r06j}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_distributed.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "bands or partitioned" > $O/pytest_dist.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_dist.log; exit 1; }
tail -1 $O/pytest_dist.log
for r in 1 2 3; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver_$r.err \
    || { echo "bench failed"; tail $O/bench_driver_$r.err; exit 1; }
  python tools/summarize_bench.py $O/bench_driver_$r.json | head -3
done
python tools/summarize_bench.py $O/bench_driver_3.json
for c in K2 K4 K5; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 0 > $O/bench_$c.json 2> $O/bench_$c.err \
    || { echo "bench $c failed"; tail $O/bench_$c.err; exit 1; }
  python tools/summarize_bench.py $O/bench_$c.json | head -2
done
timeout -k 10 300 python bench.py --side 0 --cpu-seconds 0 > $O/bench_default.json 2> $O/bench_default.err \
  || { echo "bench default failed"; tail $O/bench_default.err; exit 1; }
python tools/summarize_bench.py $O/bench_default.json | head -2
export RT_TIMELINE=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o drv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 \
  > $O/prof_line.json 2> $O/prof_line.err || { echo "rocprof failed"; tail $O/prof_line.err; exit 1; }
unset RT_TIMELINE
DB=$(find $O/prof -name "*.db" | head -1)
RT_WINDOW=$O/prof_line.json python3 tools/rocpd_stats.py $DB > $O/prof_timed_region_kernel_stats.csv || exit 1
python3 tools/rocpd_stats.py $DB > $O/prof_command_kernel_stats.csv || exit 1
cat $O/prof_timed_region_kernel_stats.csv
python -c "import json; d=json.loads(open('$O/prof_line.json').read().strip().splitlines()[-1]); print('line kernel_avg_us', d['roofline']['kernel_avg_us'], 'ms_per_step', d['ms_per_step'])"
