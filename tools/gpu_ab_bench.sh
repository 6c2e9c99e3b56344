#!/bin/bash
# Interleaved bench.py A/B of library builds: gpu_ab_bench.sh TAG "K3 K2" ROUNDS lib...
# ("default" = the in-tree build; lib:ENV=V,ENV=V adds environment).  Prints, per (config,
# round, lib), ms_per_step, the timed kernel's HIP-event average and image_ok.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; CFGS=$2; ROUNDS=$3; shift 3
O=gpurun_out/$TAG; mkdir -p $O
for c in $CFGS; do
  for r in $(seq $ROUNDS); do
    for spec in "$@"; do
      lib=${spec%%:*}; extra=""; [ "$spec" != "$lib" ] && extra=${spec#*:}
      E=""; [ $lib != default ] && E="RT_HIP_LIB=$lib"
      f=$O/${c}_${r}_$(basename $lib .so)${extra:+_${extra//[,=]/_}}.json
      env $E ${extra//,/ } timeout -k 10 300 python bench.py --config $c --side 0 \
        --cpu-seconds 0 > $f 2>> $O/bench.err || { echo "bench $c $spec failed"; tail -5 $O/bench.err; exit 1; }
      python - "$f" "$c" "$r" "$spec" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], sys.argv[3], sys.argv[4].split("/")[-1], d["ms_per_step"],
      d["roofline"]["kernel_avg_us"], d["image_ok"], flush=True)
EOF
    done
  done
done
