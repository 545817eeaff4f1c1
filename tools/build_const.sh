#!/bin/bash
# Build the working tree's libias.so with constants changed, into
# build_var/libias_NAME.so, for same-box A/B runs (tools/gpu_ab.sh).
# The variant's source is kept beside it (build_var/libias_NAME.src: HEAD,
# the working tree's diff against it and the constant edits), so a variant
# that misbehaves on the GPU can be traced after its tree is gone.
# usage: tools/build_const.sh NAME FILE 'sed-expression' [FILE 'sed-expression' ...]
#   e.g. tools/build_const.sh db4 sym2_kernels.hpp 's/SYM2_DB_MAX = 8/SYM2_DB_MAX = 4/'
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
T=/tmp/ias_const_$NAME
rm -rf $T; mkdir -p $T
cp -r include $T/
mkdir -p $T/ia-spgemm_amd
cp -r ia-spgemm_amd/csrc ia-spgemm_amd/cli ia-spgemm_amd/Makefile $T/ia-spgemm_amd/
while [ $# -ge 2 ]; do
  f=$T/ia-spgemm_amd/csrc/$1
  before=$(md5sum < $f)
  sed -i "$2" $f
  [ "$before" != "$(md5sum < $f)" ] || { echo "no change: $1 $2"; exit 1; }
  shift 2
done
{ echo "HEAD $(git rev-parse HEAD)"; echo "== working tree vs HEAD"; git diff HEAD -- include ia-spgemm_amd/csrc ia-spgemm_amd/cli;
  echo "== constant edits"; diff -ru ia-spgemm_amd/csrc $T/ia-spgemm_amd/csrc || true; } > $T/src.txt
make -C $T/ia-spgemm_amd -j8 libias.so > $T/build.log 2>&1 || { tail -20 $T/build.log; exit 1; }
mkdir -p build_var
cp $T/ia-spgemm_amd/libias.so build_var/libias_$NAME.so
cp $T/src.txt build_var/libias_$NAME.src
rm -rf $T
echo "build_var/libias_$NAME.so"
