#!/bin/bash
# Build the HIP library of git revision $1 into abtest/<rev>/librepurpose_amd.so (A/B baseline).
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
D=abtest/$REV
rm -rf "$D" && mkdir -p "$D"
git archive "$REV" repurpose_amd/csrc include Makefile | tar -x -C "$D"
make -C "$D" -j8 > "$D/build.log" 2>&1
ls -la "$D/repurpose_amd/_native/librepurpose_amd.so"
