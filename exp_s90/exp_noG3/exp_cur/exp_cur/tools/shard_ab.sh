#!/bin/bash
# Same-box overhead of the 1-rank latent-sharded step over the single-GPU step: alternating bench.py runs of
# the single-GPU step (this tree), and the sharded step of each TREE (this tree also with 2 batch slices).
#   [AB_HWQ=Q] tools/shard_ab.sh ROUNDS OUT TREE...   (every run with Q hardware queues per process, default 8)
N=$1; OUT=$2; shift 2
export GPU_MAX_HW_QUEUES=${AB_HWQ:-8}
mkdir -p "$OUT"
one() {  # tag dir args...
  local tag=$1 dir=$2; shift 2
  (cd "$dir" && timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 10 "$@") > "$OUT/${tag}_$i.json" 2> "$OUT/${tag}_$i.err" || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'])" "$OUT/${tag}_$i.json" "$tag"
}
for i in $(seq 1 "$N"); do
  one single . || exit 1
  for dir in "$@"; do
    one "sharded_$(echo "$dir" | tr '/.' '_-')" "$dir" --force-sharded || exit 1
  done
  one sharded_2slices . --force-sharded --recon-chunks 2 || exit 1
done
