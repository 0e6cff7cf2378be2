#!/usr/bin/env bash
# End of round 3: full GPU suite + smoke + a bench line per BASELINE configuration + solo C4/8
# (tools/r03_session.sh, TAG=r03g by default), then rocprofv3 kernel trace + HBM counters of C3 and C5
# (tools/profile.sh) for profiles/ and bench.py's traffic figures.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03g} bash tools/r03_session.sh || exit $?
CONFIG=c3 bash tools/profile.sh || exit $?
CONFIG=c5 STEPS=2 bash tools/profile.sh || exit $?
