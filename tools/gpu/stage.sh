#!/bin/bash
# Copy the tree as it is NOW (tracked files + the built libraries) into .gpustage/, so a queued gpurun call runs
# this consistent snapshot even if the working tree is edited while the call waits for a box.
#   bash tools/gpu/stage.sh   then   gpurun -- 'cd .gpustage && bash tools/gpu/<script>.sh'
set -e
cd "$(dirname "$0")/../.."
rm -rf .gpustage.new
mkdir -p .gpustage.new
git ls-files -z --cached --others --exclude-standard | grep -zv '^\.gpustage' | xargs -0 cp --parents -t .gpustage.new
cp --parents -t .gpustage.new kan-odes_amd/kanode/libkanode.so oracle/build/liboracle.so
for f in tools/bin/var/*.so; do [ -f "$f" ] && cp --parents -t .gpustage.new "$f"; done   # variant builds (experiments)
rm -rf .gpustage
mv .gpustage.new .gpustage
echo "staged $(git rev-parse --short HEAD) + working changes into .gpustage"
