#!/bin/bash
# Snapshot A/B on the GPU (debug tool): the random worlds named, built by this tree's library and
# by tools/ab/libketo_<variant>.so, saved and compared array by array (tools/snapdiff.py).
#   usage: tools/gpu_snapdiff.sh variant seed:rewrites...
set -u
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
V=$1; shift
O=gpurun_out/snapdiff && rm -rf $O && mkdir -p $O
timeout -k 10 120 python3 tools/snapdiff.py save $O/new "$@" || exit 1
KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$PWD/tools/ab/libketo_$V.so timeout -k 10 120 python3 tools/snapdiff.py save $O/old "$@" || exit 1
for s in "$@"; do f=$(echo $s | tr : _).bin; echo "== $s"; python3 tools/snapdiff.py compare $O/old/$f $O/new/$f; done
