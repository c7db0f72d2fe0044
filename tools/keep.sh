#!/usr/bin/env bash
# Move the last gpurun call's results into profiles/r04/<name>/ (then gpurun_out/ is empty).
set -eu
cd "$(dirname "$0")/.."
[ $# -eq 1 ] || { echo "usage: tools/keep.sh <name>"; exit 2; }
mkdir -p "profiles/r04/$1"
shopt -s dotglob nullglob
for f in gpurun_out/*; do mv "$f" "profiles/r04/$1/"; done
echo "kept in profiles/r04/$1"
