#!/bin/bash
# Builds libbloomhip from git revision REV into cs265-lsm-tree_amd/lib_alt/
# (the A side of tools/ab.sh).  Usage: tools/build_alt.sh REV
set -e
REV=${1:?rev}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/bloomhip_alt.XXXXXX)
git -C "$ROOT" worktree add -q --detach "$WT" "$REV"
trap 'git -C "$ROOT" worktree remove --force "$WT"' EXIT
OUT=$ROOT/cs265-lsm-tree_amd/lib_alt
make -C "$WT/cs265-lsm-tree_amd/csrc" -j8 OUT="$OUT" "$OUT/libbloomhip.so" > /dev/null
echo "built $OUT/libbloomhip.so from $(git -C "$ROOT" rev-parse --short "$REV")"
