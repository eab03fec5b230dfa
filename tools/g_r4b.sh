# Describe ablations in the pipelined step: base, no staging loads, no describe at all.
set -o pipefail
bash tools/ab_lib.sh 2 tum5k base dnol dnone && bash tools/ab_lib.sh 2 tum base dnol dnone
