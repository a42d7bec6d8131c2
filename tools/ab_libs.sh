#!/bin/bash
# A/B timing of alternative engine builds in tools/ab/ on C3 (and the current build)
cd "$(dirname "$0")/.."
for lib in cur tools/ab/libketo_*.so; do
  if [ "$lib" = cur ]; then unset KETO_MI355X_LIB_OVERRIDE KETO_MI355X_ALLOW_OVERRIDE; name=cur
  else export KETO_MI355X_ALLOW_OVERRIDE=tools KETO_MI355X_LIB_OVERRIDE=$PWD/$lib; name=$(basename $lib); fi
  timeout -k 10 120 python3 tools/build_scale.py --scale ${SCALE:-1} --batches 4 2>&1 | grep -E "batch 3|allowed" | sed "s/^/$name: /" || exit 1
done
