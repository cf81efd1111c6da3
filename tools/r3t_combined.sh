#!/bin/bash
# Copy-split / non-temporal pack A/B of the streamed calls, then the round-3
# profiles (tools/r3r_profile.sh).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/r3s_parts.sh || exit $?
bash tools/r3r_profile.sh || exit $?
