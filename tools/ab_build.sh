#!/bin/bash
# A/B builds of the Check interpreter (tool, not product): tools/ab/libketo_<name>.so, each
# the engine library with one kernel source (default csrc/check.hip) compiled under extra -D flags.
#   usage: tools/ab_build.sh name "-DKETO_RING=4 -DKETO_GUARD=24" [check.hip source]
set -eu
cd "$(dirname "$0")/../djy-keto_amd"
make -s -j8 >/dev/null
NAME=$1; FLAGS=$2; SRC=${3:-csrc/check.hip}
mkdir -p ../tools/ab build/ab
BASE=$(basename $SRC .hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Icsrc $FLAGS -c $SRC -o build/ab/${BASE}_$NAME.o
OBJS=$(ls build/*.o | grep -v "/$BASE.o\$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../tools/ab/libketo_$NAME.so $OBJS build/ab/${BASE}_$NAME.o -lpthread
echo built tools/ab/libketo_$NAME.so
