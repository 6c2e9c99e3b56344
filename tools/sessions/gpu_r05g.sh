#!/bin/bash
# Round 5, session g: the committed build (the accumulator's Markstein division) — the GPU
# suite and smoke; the 8-rank K3 chain share's call under a kernel + HIP runtime trace
# (which HIP calls the host makes before the launch reaches the GPU).
# Usage: bash tools/sessions/gpu_r05g.sh TAG
set -o pipefail
TAG=${1:-r05g}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace -f csv -d $O/tl_s8 -o tl -- python3 tools/share_region.py 8 0 5 20 \
  > $O/tl_s8_line.json 2> $O/tl_s8.err || { echo "rocprof s8 failed"; tail $O/tl_s8.err; exit 1; }
python tools/timeline.py $O/tl_s8 $O/tl_s8_line.json > $O/timeline_s8.json || exit 1
python -c "import json; d=json.load(open('$O/timeline_s8.json')); print(json.dumps({k: v for k, v in d.items() if k != 'kernels'})[:3000])"
timeout -k 10 120 python tools/share_region.py 8 0 15 20 > $O/share_n8.json 2> $O/share_n8.err || { tail $O/share_n8.err; exit 1; }
python -c "import json; d=json.load(open('$O/share_n8.json')); d.pop('timeline_host'); print(d)"
