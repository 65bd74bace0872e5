#!/bin/bash
# Round-3 pass ae: kernel stats + FETCH / WRITE PMC of the final build's
# stereo (1024 pairs, left LSD split) and rig (512 cameras) legs.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
MODE=kitti bash tools/prof.sh r03ae_kitti || exit 1
MODE=rig bash tools/prof.sh r03ae_rig || exit 1
