# Marginal cost of each extraction stage in the pipelined step: stage k launched twice.
set -o pipefail
bash tools/ab_envp.sh 2 tum - ORBX_DUP_STAGE=1 ORBX_DUP_STAGE=2 ORBX_DUP_STAGE=3 ORBX_DUP_STAGE=4 ORBX_DUP_STAGE=5 && \
bash tools/ab_envp.sh 1 tum5k - ORBX_DUP_STAGE=1 ORBX_DUP_STAGE=2 ORBX_DUP_STAGE=3 ORBX_DUP_STAGE=4 ORBX_DUP_STAGE=5
