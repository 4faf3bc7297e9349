#!/bin/bash
# A/B of the attention backward's persistent-grid cap (DGPPO_BWD2_BLOCKS) on one minibatch's Vl pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for b in 1024 512 2048 4096 1024; do
  DGPPO_BWD2_BLOCKS=$b timeout -k 10 120 python3 scripts/ab_passes.py || exit 1
done
