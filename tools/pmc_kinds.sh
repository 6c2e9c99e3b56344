#!/bin/bash
# Issue/stall counter groups per trace-kernel instance over tools/time_kernel.py CFG (single-
# frame updates + fused launches), one rocprofv3 --pmc pass per group.
# Usage: bash tools/pmc_kinds.sh TAG CFG LIB "kernel-substr ..."
set -o pipefail
TAG=$1; CFG=$2; LIB=$3; KS=$4
cd $GRAFT_REPO_ROOT; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp RT_HIP_LIB=$GRAFT_REPO_ROOT/$LIB
n=$(basename $LIB .so)
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
G2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INST_CYCLES_VMEM"
files=""
for g in 1 2; do
  eval "CS=\$G$g"
  timeout -k 10 180 rocprofv3 --pmc $CS --output-format csv -d $O/raw -o ${n}_${CFG}_g$g -- python3 tools/time_kernel.py $CFG > $O/log_${n}_${CFG}_g$g.txt 2>&1 || { echo "pmc g$g failed"; tail -5 $O/log_${n}_${CFG}_g$g.txt; exit 1; }
  files="$files $O/raw/${n}_${CFG}_g${g}_counter_collection.csv"
done
for k in $KS; do
  python3 tools/pmc_summary.py $O/pmc_${n}_${CFG}_$k.json "$k" $files > /dev/null
  python3 -c "
import json; d=json.load(open('$O/pmc_${n}_${CFG}_$k.json')); m=d['median_per_launch']; w=m.get('SQ_WAVES',1)
print('$n $CFG $k', 'waves', w, {k: round(v/w,1) for k,v in m.items() if k!='SQ_WAVES'}, 'gui', m.get('GRBM_GUI_ACTIVE'))"
done
