#!/bin/bash
# A/B baselines: export git revision REV (default HEAD) into DIR (default ab_base/; git-ignored,
# travels to the GPU box with the snapshot) and build its library there, so that
# `python3 DIR/bench.py ...` and `python3 bench.py ...` can alternate on one box (tools/ab_tree.sh).
set -euo pipefail
REV=${1:-HEAD}
DIR=${2:-ab_base}
cd "$(dirname "$0")/.."
case "$DIR" in ab_*) ;; *) echo "DIR must start with ab_" >&2; exit 1 ;; esac
rm -rf "$DIR" && mkdir "$DIR"
git archive "$REV" | tar -x -C "$DIR"
make -C "$DIR/mpc-verde_amd" -j8 >/dev/null 2>&1
make -C "$DIR/oracle" >/dev/null 2>&1
echo "$DIR: $(git rev-parse --short "$REV")"
