#!/bin/bash
# Round 6 closing measurements of the final tree (after the accumulation micro-cuts, the
# hit records through buffer loads and the min3 domain checks): the whole GPU suite, smoke, the driver's K3 command three
# times, --config K2 / K4 / K5, the default length, the driver's command under rocprofv3
# --kernel-trace --stats with the timed region's host stamps (RT_TIMELINE=1;
# tools/rocpd_stats.py RT_WINDOW), and the K3 and K5 PMC passes (tools/pmc_bench.sh) for
# pmc_r06_K3.json / pmc_r06_K5.json.
set -o pipefail
TAG=${1:-r06be}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2 3; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver_$r.err \
    || { echo "bench failed"; tail $O/bench_driver_$r.err; exit 1; }
  python tools/summarize_bench.py $O/bench_driver_$r.json > $O/summary_driver_$r.txt; head -1 $O/summary_driver_$r.txt
done
for c in K2 K4 K5; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 0 > $O/bench_$c.json 2> $O/bench_$c.err \
    || { echo "bench $c failed"; tail $O/bench_$c.err; exit 1; }
  python tools/summarize_bench.py $O/bench_$c.json > $O/summary_$c.txt; head -1 $O/summary_$c.txt
done
timeout -k 10 300 python bench.py --side 0 --cpu-seconds 0 > $O/bench_default.json 2> $O/bench_default.err \
  || { echo "bench default failed"; tail $O/bench_default.err; exit 1; }
python tools/summarize_bench.py $O/bench_default.json > $O/summary_default.txt; head -1 $O/summary_default.txt
export RT_TIMELINE=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o drv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --side 0 --cpu-seconds 0 \
  > $O/prof_line.json 2> $O/prof_line.err || { echo "rocprof failed"; tail $O/prof_line.err; exit 1; }
unset RT_TIMELINE
DB=$(find $O/prof -name "*.db" | head -1)
RT_WINDOW=$O/prof_line.json python3 tools/rocpd_stats.py $DB > $O/prof_timed_region_kernel_stats.csv || exit 1
python3 tools/rocpd_stats.py $DB > $O/prof_command_kernel_stats.csv || exit 1
cat $O/prof_timed_region_kernel_stats.csv
PMC_ROUND=r06 bash tools/pmc_bench.sh $TAG "K3" > $O/pmc.log 2>&1 || { echo "pmc failed"; tail $O/pmc.log; exit 1; }
ls $O/pmc_r06_K3.json
PMC_ROUND=r06 bash tools/pmc_bench.sh $TAG "K5" > $O/pmc_k5.log 2>&1 || { echo "pmc K5 failed"; tail $O/pmc_k5.log; exit 1; }
ls $O/pmc_r06_K5.json
