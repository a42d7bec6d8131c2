#!/bin/bash
# Measurement-only variant of one kernel source (no emulated parity gate, unlike ab_build.sh):
# tools/ab/libketo_<name>.so = the engine library with SRC compiled under extra -D flags.
#   usage: tools/ab_variant.sh name "-DKETO_FR_NOTAB" [csrc/frontier.hip]
set -eu
cd "$(dirname "$0")/../djy-keto_amd"
make -s -j8 >/dev/null
NAME=$1; FLAGS=$2; SRC=${3:-csrc/frontier.hip}
mkdir -p ../tools/ab build/ab
BASE=$(basename $SRC .hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Icsrc $FLAGS -c $SRC -o build/ab/${BASE}_$NAME.o
OBJS=$(ls build/*.o | grep -v "/$BASE.o\$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../tools/ab/libketo_$NAME.so $OBJS build/ab/${BASE}_$NAME.o -lpthread
echo built tools/ab/libketo_$NAME.so
