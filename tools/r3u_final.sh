#!/bin/bash
# Copy-split / non-temporal pack A/B of the streamed calls, then the
# driver's round-end sequence (full -m gpu suite, smoke, default bench).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/r3s_parts.sh || exit $?
bash tools/round_check.sh || exit $?
