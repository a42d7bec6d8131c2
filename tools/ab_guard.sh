#!/bin/bash
# A/B: Check interpreter pseudo-step budget per load slot (KETO_CHECK_GUARD) on C3
cd "$(dirname "$0")/.."
for g in 24 12 6 3; do
  KETO_CHECK_GUARD=$g timeout -k 10 120 python3 tools/build_scale.py --scale 1 --batches 4 2>&1 | grep -E "batch 3|allowed" | sed "s/^/guard $g: /" || exit 1
done
