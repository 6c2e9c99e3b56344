#!/bin/bash
# Round 5, session q: concurrent parts per one-frame update in the driver's region on the
# current host path (CPython binding, fork skip): 2 (AUTO) / 3 / 4, interleaved in one
# process, K3 and K2, twice.
# Usage: bash tools/sessions/gpu_r05q.sh TAG
set -o pipefail
TAG=${1:-r05q}
cd $GRAFT_REPO_ROOT; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in K3 K2; do
    timeout -k 10 200 python tools/driver_region.py 25 $cfg "q2=;queues=2" "q3=;queues=3" "q4=;queues=4" > $O/region_${cfg}_$r.jsonl 2> $O/region_${cfg}_$r.err \
      || { tail $O/region_${cfg}_$r.err; exit 1; }
    python -c "
import json
for l in open('$O/region_${cfg}_$r.jsonl'):
    d = json.loads(l); print('$cfg', d['variant'], 'wall', d['wall_us_per_step_q1_med_q3'], 'ev', d['events_us_per_step_q1_med_q3'], 'issue', d['issue_us_q1_med_q3'])"
  done
done
