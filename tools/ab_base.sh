#!/bin/bash
# Build the library of a git revision (default HEAD) into build/variants/liblsr_base.so for
# same-box A/B runs against the working tree (tools/gpu.sh ab benches the variants).
set -e
rev=${1:-HEAD}
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" 4dlangsplat_amd/csrc include | tar -x -C "$tmp"
make -s -j8 -C "$tmp/4dlangsplat_amd/csrc"
mkdir -p "$root/4dlangsplat_amd/build/variants"
cp "$tmp/4dlangsplat_amd/build/liblsr.so" "$root/4dlangsplat_amd/build/variants/liblsr_base.so"
rm -rf "$tmp"
echo "built variants/liblsr_base.so from $rev"
