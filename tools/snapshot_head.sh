#!/bin/bash
# Build tree of a commit (default HEAD) for tools/ab_trees.sh: exp_head/ (sources + its own library, no fixtures)
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rm -rf "$ROOT/exp_head" && mkdir -p "$ROOT/exp_head"
git -C "$ROOT" archive "$REV" | tar -x -C "$ROOT/exp_head" --exclude=tests/golden
make -s -C "$ROOT/exp_head/crosscoder-model-diff-replication_amd/csrc" -j8 > /dev/null
echo "$ROOT/exp_head"
