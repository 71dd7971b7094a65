#!/bin/bash
# variant_rev.sh <tag> <git-rev> [-DFLAG ...]: build libbrc_hip.so from the sources of <git-rev> (a
# throwaway worktree) into ab/<tag>/ -- the A/B baseline of tools/ab.sh (dev tool)
set -e
TAG=$1; REV=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=/tmp/brc_wt_$TAG
rm -rf $WT; git -C $ROOT worktree prune
git -C $ROOT worktree add --detach $WT $REV >/dev/null
python3 $WT/tools/variant.py $TAG "$@" >/dev/null
mkdir -p $ROOT/ab/$TAG
cp $WT/ab/$TAG/libbrc_hip.so $ROOT/ab/$TAG/libbrc_hip.so 2>/dev/null || cp $WT/exp/$TAG/libbrc_hip.so $ROOT/ab/$TAG/libbrc_hip.so   # revisions before round 5 build into exp/
git -C $ROOT worktree remove --force $WT
echo $ROOT/ab/$TAG/libbrc_hip.so
