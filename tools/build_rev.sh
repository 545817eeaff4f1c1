#!/bin/bash
# Build libias.so of git revision REV (default HEAD) into build_var/libias_NAME.so,
# for same-box A/B runs against the working tree (tools/gpu_ab.sh).
# usage: tools/build_rev.sh NAME [REV]
set -e
cd "$(dirname "$0")/.."
NAME=$1; REV=${2:-HEAD}
WT=/tmp/ias_wt_$NAME
rm -rf $WT
git worktree prune
git worktree add -f --detach $WT $REV > /dev/null
make -C $WT/ia-spgemm_amd -j8 libias.so > /dev/null 2>&1
mkdir -p build_var
cp $WT/ia-spgemm_amd/libias.so build_var/libias_$NAME.so
echo "REV $(git rev-parse $REV)" > build_var/libias_$NAME.src   # the variant's source: that revision
git worktree remove --force $WT
echo "build_var/libias_$NAME.so <- $(git rev-parse --short $REV)"
