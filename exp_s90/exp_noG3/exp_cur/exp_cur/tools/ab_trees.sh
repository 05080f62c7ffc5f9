#!/bin/bash
# Same-box A/B of two source trees (each with its own built library): alternating bench.py runs.
#   tools/ab_trees.sh OLD_TREE NEW_TREE ROUNDS OUT   (OLD_TREE e.g. exp_head/ from tools/snapshot_head.sh)
OLD=$1; NEW=$2; N=${3:-4}; OUT=${4:-gpurun_out/ab_trees}
mkdir -p "$OUT"
for i in $(seq 1 "$N"); do
  for t in old new; do
    dir=$OLD; [ $t = new ] && dir=$NEW
    (cd "$dir" && timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 10) > "$OUT/${t}_$i.json" 2> "$OUT/${t}_$i.err" || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'])" "$OUT/${t}_$i.json" $t
  done
done
