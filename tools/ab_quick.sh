#!/bin/bash
# A/B builds that change only scheduling knobs (waves per SIMD, block sizes), not semantics (tool,
# not product): tools/ab/libketo_<name>.so = the engine library with one kernel source compiled
# under extra -D flags, without tools/ab_build.sh's emulated parity pass.
#   usage: tools/ab_quick.sh name "-DKETO_FR_WAVES0=5" [csrc/frontier.hip]
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
