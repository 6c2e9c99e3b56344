#!/bin/bash
# Issue/stall counters of the trace kernel over tools/time_kernel.py, one rocprofv3 --pmc
# pass per counter group (no trace domains with --pmc).  Usage: bash tools/pmc_kernel.sh
# TAG "k3 k2" [lib.so]  -> gpurun_out/TAG/pmc_<cfg>.json
set -o pipefail
TAG=$1; CFGS=$2; LIB=${3:-}
cd $GRAFT_REPO_ROOT; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
[ -n "$LIB" ] && export RT_HIP_LIB=$GRAFT_REPO_ROOT/$LIB
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
G2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VALU_TRANS_F32"
G3="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_CVT SQ_INST_CYCLES_SMEM"
for c in $CFGS; do
  files=""
  for g in 1 2 3; do
    eval "CS=\$G$g"
    timeout -k 10 180 rocprofv3 --pmc $CS --output-format csv -d $O/pmc_raw -o ${c}_g$g -- python3 tools/time_kernel.py $c > $O/pmc_${c}_g$g.log 2>&1 || { echo "pmc $c g$g failed"; tail -5 $O/pmc_${c}_g$g.log; exit 1; }
    files="$files $(ls $O/pmc_raw/${c}_g${g}_counter_collection.csv)"
  done
  python3 tools/pmc_summary.py $O/pmc_$c.json trace_kernel $files > /dev/null && echo "== $c" && python3 -c "
import json; d=json.load(open('$O/pmc_$c.json')); m=d['median_per_launch']; w=m['SQ_WAVES']
print({k: round(v/w,1) for k,v in m.items()})"
done
