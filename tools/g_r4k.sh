# Upper bound of reading level 0 in place: the pyramid's level-0 copy skipped (timing only).
set -o pipefail
STEPS=50 bash tools/ab_lib.sh 3 tum base nol0 && STEPS=30 bash tools/ab_lib.sh 2 tum5k base nol0
