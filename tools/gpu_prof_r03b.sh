#!/bin/bash
# round-3 PMC passes of the lines leg and of the headline with the map model
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
MODE=lines bash tools/prof.sh lines_r03 || exit 1
MODE=points bash tools/prof.sh points_r03b || exit 1
echo all ok
