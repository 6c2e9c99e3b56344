#!/bin/bash
# Round 6 final check, as the round-end driver runs it on a tree built from scratch
# (make clean + __graft_entry__.build() here): the whole GPU suite, smoke, bench.py with no
# arguments and with the driver's --gpus 1 --steps 20 --warmup 5, then the N > 1 rehearsal
# over gloo (tools/gpu_rehearse.sh: 2-4 ranks sharing the GPU, images checked).
set -o pipefail
TAG=${1:-r06bg}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_noargs.json 2> $O/bench_noargs.err \
  || { echo "bench failed"; tail $O/bench_noargs.err; exit 1; }
python tools/summarize_bench.py $O/bench_noargs.json | head -1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
  || { echo "bench failed"; tail $O/bench_driver.err; exit 1; }
python tools/summarize_bench.py $O/bench_driver.json | head -1
bash tools/gpu_rehearse.sh $TAG/rehearse > $O/rehearse.log 2>&1 || { echo "rehearse failed"; tail $O/rehearse.log; exit 1; }
cat $O/rehearse.log
