#!/bin/bash
# Round 3 re-entry: the driver's round-end sequence on the current code, then
# the download-pattern decode legs and the per-stripe descriptor bench.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/round_check.sh || exit $?
bash tools/r3e_check.sh || exit $?
