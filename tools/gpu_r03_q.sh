#!/bin/bash
# Round-3 pass q: profiles of the split build (points headline + lines):
# kernel trace + stats, FETCH / WRITE PMC passes (tools/prof.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
MODE=points bash tools/prof.sh r03q_points || exit 1
MODE=lines bash tools/prof.sh r03q_lines || exit 1
