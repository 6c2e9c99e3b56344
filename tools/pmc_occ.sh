#!/bin/bash
# Occupancy / issue counters of the trace kernel over tools/time_kernel.py (one --pmc pass).
# Usage: bash tools/pmc_occ.sh TAG CFG [lib.so ...]  -> gpurun_out/TAG/occ_<lib>_<cfg>.json
set -o pipefail
TAG=$1; CFG=$2; shift 2
cd $GRAFT_REPO_ROOT; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
CS="SQ_LEVEL_WAVES SQ_CYCLES SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
for L in "$@"; do
  n=$(basename $L .so)
  RT_HIP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 180 rocprofv3 --pmc $CS --output-format csv -d $O/raw -o ${n}_$CFG -- python3 tools/time_kernel.py $CFG > $O/log_${n}_$CFG.txt 2>&1 || { echo "pmc $n failed"; tail -5 $O/log_${n}_$CFG.txt; exit 1; }
  python3 tools/pmc_summary.py $O/occ_${n}_$CFG.json trace_kernel $O/raw/${n}_${CFG}_counter_collection.csv > /dev/null
  python3 -c "
import json; d=json.load(open('$O/occ_${n}_$CFG.json')); m=d['median_per_launch']
print('$n', {k: round(v) for k, v in m.items()}, 'level/cycles', round(m['SQ_LEVEL_WAVES']/m['SQ_CYCLES'], 3), 'level/busy', round(m['SQ_LEVEL_WAVES']/m['SQ_BUSY_CYCLES'], 3))"
done
