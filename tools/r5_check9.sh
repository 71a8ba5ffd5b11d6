#!/bin/bash
# Null-refine tests + the refine-cost profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash tools/r5_check8.sh || exit $?
bash tools/r5_refine.sh
