#!/bin/bash
# quick tests + lv4096 trace, then the anchors
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu/r6_quick.sh || exit 3
bash tools/gpu/r6_anchors.sh || exit 3
