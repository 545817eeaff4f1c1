#!/bin/bash
# Copy the working tree's built libias.so to build_var/libias_NAME.so for a
# same-box A/B (tools/gpu_ab.sh), with its source kept beside it
# (build_var/libias_NAME.src: HEAD and the working tree's diff against it).
# usage: tools/build_cur.sh NAME
set -e
cd "$(dirname "$0")/.."
NAME=$1
make -C ia-spgemm_amd -j8 libias.so > /dev/null
mkdir -p build_var
cp ia-spgemm_amd/libias.so build_var/libias_$NAME.so
{ echo "HEAD $(git rev-parse HEAD)"; git diff HEAD -- include ia-spgemm_amd/csrc ia-spgemm_amd/cli; } > build_var/libias_$NAME.src
echo "build_var/libias_$NAME.so"
