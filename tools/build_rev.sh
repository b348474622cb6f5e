#!/usr/bin/env bash
# Build libkanode.so of a git revision (A/B reference):  tools/build_rev.sh REV NAME -> tools/bin/var/NAME.so
set -eu
cd "$(dirname "$0")/.."
rev=$1; name=$2
wt=/tmp/kanode_rev_$name
rm -rf $wt; git worktree prune
git worktree add --detach $wt $rev > /dev/null
make -C $wt/kan-odes_amd -j8 > /tmp/build_rev_$name.log 2>&1
mkdir -p tools/bin/var
cp $wt/kan-odes_amd/kanode/libkanode.so tools/bin/var/$name.so
git worktree remove --force $wt
echo built tools/bin/var/$name.so from $(git rev-parse --short $rev)
