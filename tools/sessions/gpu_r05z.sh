#!/bin/bash
# Round 5, closing session: the committed tree's evidence — the GPU suite and smoke; the
# driver's command three times and the default length; the command under rocprofv3
# --kernel-trace --stats (per-kernel summary); the region's gated kernel trace with host
# stamps (tools/timeline.py: the per-update union the roofline's kernel time is checked
# against); the PMC passes of the timed K3 kernel at the timed structure (two parts).
# Usage: bash tools/sessions/gpu_r05z.sh TAG
set -o pipefail
TAG=${1:-r05z}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.json 2> $O/bench_driver_$r.err \
    || { echo bench failed; tail $O/bench_driver_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_driver_$r.json')); r=d['roofline']; s=d['rank_shares']['K3']; print('driver', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'], 'k2', d['k2']['us_per_step'], 'chain8', s['chain']['8']['us_per_step'], s['chain']['8']['efficiency_vs_1gpu_step'])"
done
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err \
  || { echo bench failed; tail $O/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_default.json')); r=d['roofline']; print('default', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['image_ok'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_driver -o driver -- python3 bench.py --gpus 1 --steps 20 --warmup 5 \
  > $O/prof_driver.log 2>&1 || { echo "rocprof failed"; tail $O/prof_driver.log; exit 1; }
echo rocprof done
RT_TIMELINE=1 timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/tl_g20 -o tl -- python3 bench.py --gpus 1 --gate --steps 20 --warmup 5 --side 0 --cpu-seconds 0 \
  > $O/tl_g20_line.json 2> $O/tl_g20.err || { echo "rocprof g20 failed"; tail $O/tl_g20.err; exit 1; }
python tools/timeline.py $O/tl_g20 $O/tl_g20_line.json > $O/timeline_g20.json || exit 1
python -c "import json; d=json.load(open('$O/timeline_g20.json')); [d.pop(k) for k in ('hip_calls','kernels')]; print('g20', json.dumps(d))"
PMC_ROUND=r05 QUEUES=0 bash tools/pmc_bench.sh ${TAG}_pmc "K3 K2" || exit 1
echo pmc done
