#!/bin/bash
# PMC summaries of the timed trace kernel of `bench.py --config CFG` (the kernel instance and
# frames per launch the bench line reports): FETCH_SIZE and WRITE_SIZE in separate passes
# (MI355X_MICROARCH.md §HBM), then SQ/GRBM groups and the VALU instruction classes (two
# passes of 8 SQ counters, read by tools/valu_weighted.py).  Writes gpurun_out/TAG/pmc_${PMC_ROUND}_CFG.json
# (copy to profiles/ to have bench.py report `traffic` and `roofline.valu` from it).
# QUEUES (default 0 = the library's choice, what bench.py times: two concurrent half-image
# parts per K3 update) is passed as --queues; the summary records it, and bench.py scales the
# per-launch counts by it (one update = QUEUES launches of equal halves).
# K2/K3 run the driver's --steps 20 --warmup 5 (the timed chain is one 20-frame launch: the
# summary's frames_per_launch must match the line's).
# Usage: [PMC_ROUND=r06] [QUEUES=0] bash tools/pmc_bench.sh TAG "K3 K2 K4 K5"
set -o pipefail
TAG=$1; CFGS=$2; PMC_ROUND=${PMC_ROUND:-r06}; QUEUES=${QUEUES:-0}
cd $GRAFT_REPO_ROOT; O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for c in $CFGS; do
  ARGS="--config $c --side 0 --cpu-seconds 0 --queues $QUEUES"
  [ "$c" = "K5" ] && ARGS="$ARGS --steps 1 --warmup 1"
  { [ "$c" = "K3" ] || [ "$c" = "K2" ]; } && ARGS="$ARGS --steps 20 --warmup 5"
  timeout -k 10 300 python3 bench.py $ARGS > $O/pmc_bench_$c.json 2> $O/pmc_bench_$c.err \
    || { echo "bench $c failed"; tail -3 $O/pmc_bench_$c.err; exit 1; }
  K=$(python3 -c "import json; print(json.loads(open('$O/pmc_bench_$c.json').read())['roofline']['kernel'])")
  F=$(python3 -c "import json; print(json.loads(open('$O/pmc_bench_$c.json').read())['roofline']['frames_per_launch'])")
  i=0
  for CS in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
            "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64" \
            "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_WAVES"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $CS --output-format csv -d $O/raw -o ${c}_p$i -- python3 bench.py $ARGS \
      > $O/pmc_${c}_p$i.log 2>&1 || { echo "pmc $c pass $i failed"; tail -5 $O/pmc_${c}_p$i.log; exit 1; }
  done
  U=$(python3 -c "import json; print(json.loads(open('$O/pmc_bench_$c.json').read())['roofline']['kernel_avg_us'])")
  Q=$(python3 -c "import json; print(json.loads(open('$O/pmc_bench_$c.json').read())['roofline']['queues'])")
  PMC_QUEUES=$Q python3 tools/pmc_bench_summary.py $O/pmc_${PMC_ROUND}_$c.json "$K" "$F" $O/raw/${c}_p*_counter_collection.csv \
    || exit 1
  python3 -c "import json; d=json.load(open('$O/pmc_${PMC_ROUND}_$c.json')); d['kernel_avg_us']=$U; json.dump(d, open('$O/pmc_${PMC_ROUND}_$c.json','w'), indent=1)"
done
