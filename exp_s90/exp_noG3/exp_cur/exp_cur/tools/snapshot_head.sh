#!/bin/bash
# Build tree of a commit (default HEAD) for tools/ab_trees.sh / ab_multi.sh: DIR (default exp_head/; sources +
# its own library, no fixtures).   tools/snapshot_head.sh [REV] [DIR]
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
DIR=$ROOT/${2:-exp_head}
rm -rf "$DIR" && mkdir -p "$DIR"
git -C "$ROOT" archive "$REV" | tar -x -C "$DIR" --exclude=tests/golden
make -s -C "$DIR/crosscoder-model-diff-replication_amd/csrc" -j8 > /dev/null
echo "$DIR"
