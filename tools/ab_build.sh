#!/bin/bash
# A/B builds of the Check interpreter (tool, not product): tools/ab/libketo_<name>.so, each
# the engine library with one kernel source (default csrc/check.hip) compiled under extra -D flags.
# Every variant first passes the parity subset under the CPU emulation built with the same flags
# (tools/cpuemu, one transition per step): a variant that is wrong there never reaches a GPU.
#   usage: tools/ab_build.sh name "-DKETO_RING=4 -DKETO_GUARD=24" [check.hip source]
set -eu
cd "$(dirname "$0")/../djy-keto_amd"
make -s -j8 >/dev/null
NAME=$1; FLAGS=$2; SRC=${3:-csrc/check.hip}
mkdir -p ../tools/ab build/ab
EMU=/tmp/ab_emu_$NAME
make -s -j8 -C ../tools/cpuemu OBJDIR=$EMU/obj LIB=$EMU/lib.so "OPT=-O1 -DKETO_GUARD=1 $FLAGS" >/dev/null
(cd .. && KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$EMU/lib.so timeout 900 python3 -m pytest -q -x -m gpu \
  -p no:cacheprovider tests/test_gpu_parity.py -k "golden or random_worlds or synthetic_small" > $EMU/parity.log 2>&1) \
  || { echo "variant $NAME fails the emulated parity suite:"; tail -5 $EMU/parity.log; exit 1; }
BASE=$(basename $SRC .hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Icsrc $FLAGS -c $SRC -o build/ab/${BASE}_$NAME.o
OBJS=$(ls build/*.o | grep -v "/$BASE.o\$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../tools/ab/libketo_$NAME.so $OBJS build/ab/${BASE}_$NAME.o -lpthread
echo built tools/ab/libketo_$NAME.so "(emulated parity: $(tail -1 $EMU/parity.log))"
