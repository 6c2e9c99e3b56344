#!/bin/bash
# PMC of the K3 8-rank share's 20-frame launch (rank 0; four waves per tile, AUTO's choice,
# and four per tile pair) beside the whole image's (tools/pmc_share.py): VALU instructions
# and the SQ's busy / wave / wait cycles per pixel-frame, to tell the share's 42 % higher
# per-frame cost apart between more instructions and idle issue slots.
set -o pipefail
TAG=${1:-r06ap}
cd $GRAFT_REPO_ROOT; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for run in "8 quad rt_trace_kernel<4>" "8 quad2 rt_tpair_kernel<4>" "1 auto rt_tpair_kernel<2>"; do
  set -- $run
  n=$1; m=$2; k=$3; i=0
  for CS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
            "SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $CS --output-format csv -d $O/raw -o n${n}_${m}_p$i -- python3 tools/pmc_share.py $n 0 $m \
      > $O/pmc_n${n}_${m}_p$i.log 2>&1 || { echo "pmc $n $m pass $i failed"; tail -5 $O/pmc_n${n}_${m}_p$i.log; exit 1; }
  done
  python3 tools/pmc_bench_summary.py $O/pmc_share_n${n}_${m}.json "$k" 20 $O/raw/n${n}_${m}_p*_counter_collection.csv || exit 1
done
