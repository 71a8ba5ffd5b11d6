#!/bin/bash
# Same-box A/B: side streams (delayed-null mask table) at the lowest stream
# priority vs the product (default priority): the 256-channel share and C3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
AB_ARGS="--nchan 256" bash tools/r3_abn.sh prio256 "prod=- lowp=psrsigsim_amd/libpss_hip_lowprio.so" skip-tests || exit $?
AB_ARGS="" bash tools/r3_abn.sh prioc3 "prod=- lowp=psrsigsim_amd/libpss_hip_lowprio.so" skip-tests || exit $?
