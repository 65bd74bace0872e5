#!/bin/bash
# Round-4 pass c: kernel trace + FETCH / WRITE PMC + two SQ passes of the
# headline (points, 1024 streams) and trace + PMC of the lines leg (3072).
set -o pipefail
MODE=points SQ=1 SQ2=1 bash tools/prof.sh r04_points || exit 1
MODE=lines bash tools/prof.sh r04_lines || exit 1
exit 0
