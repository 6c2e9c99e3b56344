#!/bin/bash
# Round 6: frame-group modes re-measured on the final kernels (after the late cuts of
# DESIGN §4.3): rank 0's K3 share at 8, 4 and 2 ranks, 20-frame chain calls, modes quad
# (rt_trace_kernel<4>), quad2 (rt_tpair_kernel<4>) and on2 (rt_tpair_kernel<2>)
# alternating call by call (tools/pairs_ab.py) — does AUTO's choice still hold?
set -o pipefail
TAG=${1:-r06bd}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python tools/pairs_ab.py 15 8,4,2 quad,quad2,on2 20 every > $O/modes.jsonl 2> $O/modes.err \
  || { echo "pairs_ab failed"; tail $O/modes.err; exit 1; }
cat $O/modes.jsonl
