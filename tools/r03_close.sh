#!/bin/bash
# Round-3 closing check of the final tree: parity suite, smoke, bench (CPU baselines),
# rocprofv3 kernel stats, real-frame bench + stats, c3 and c5 bench lines.
set -o pipefail
tag=${1:-r03zc}
bash tools/final_check.sh $tag || exit 1
bash tools/r03_measure.sh $tag fixup,c3,c5
