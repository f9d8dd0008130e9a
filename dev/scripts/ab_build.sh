#!/bin/bash
# Build the extension at git revision REV into ab/_C_REV.so (for same-box A/B timing with
# TDL_EXT_SO=ab/_C_REV.so), leaving the working tree's own build untouched.
#   bash dev/scripts/ab_build.sh REV
set -e
rev=$1
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d /tmp/tdl_ab.XXXX)
git -C "$root" worktree add --detach "$tmp" "$rev" > /dev/null
(cd "$tmp" && python build_ext.py > /dev/null)
mkdir -p "$root/ab"
cp "$tmp"/tensorflowdistributedlearning_amd/_C*.so "$root/ab/_C_$rev.so"
git -C "$root" worktree remove --force "$tmp"
echo "$root/ab/_C_$rev.so"
