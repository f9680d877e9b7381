#!/bin/bash
# A/B baseline: export git revision REV (default HEAD) into ab_base/ (git-ignored, travels to the
# GPU box with the snapshot) and build its library there, so `python3 ab_base/bench.py ...` and
# `python3 bench.py ...` can alternate on one box (tools/ab_tree.sh).
set -euo pipefail
REV=${1:-HEAD}
cd "$(dirname "$0")/.."
rm -rf ab_base && mkdir ab_base
git archive "$REV" | tar -x -C ab_base
make -C ab_base/mpc-verde_amd -j8 >/dev/null 2>&1
make -C ab_base/oracle >/dev/null 2>&1
echo "ab_base: $(git rev-parse --short "$REV")"
