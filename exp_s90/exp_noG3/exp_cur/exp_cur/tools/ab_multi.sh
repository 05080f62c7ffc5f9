#!/bin/bash
# Same-box A/B/C of several source trees (each with its own built library): alternating bench.py runs.
#   [AB_ARGS="--force-sharded ..."] tools/ab_multi.sh ROUNDS OUT TREE...   (trees from tools/snapshot_head.sh, "." = this tree)
N=$1; OUT=$2; shift 2
mkdir -p "$OUT"
for i in $(seq 1 "$N"); do
  for dir in "$@"; do
    tag=$(echo "$dir" | tr '/.' '_-')
    (cd "$dir" && timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 10 $AB_ARGS) > "$OUT/${tag}_$i.json" 2> "$OUT/${tag}_$i.err" || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'])" "$OUT/${tag}_$i.json" "$dir"
  done
done
