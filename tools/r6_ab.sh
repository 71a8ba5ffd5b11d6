#!/bin/bash
# Round-6 GPU step: full GPU suite with the product library, then a same-box
# A/B of C3 bench lines (tools/r3_abn.sh: product vs variant builds).
# usage: tools/r6_ab.sh TAG "name=lib ..." [skip-tests]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
mkdir -p gpurun_out/r06
exec_ab() { AB_STEPS=${AB_STEPS:-20} bash tools/r3_abn.sh "$@"; }
exec_ab "$1" "$2" "$3"
