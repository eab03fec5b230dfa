# k_pyramid level-0 tile size now that level 0 is not stored (configs[1], pipelined, bit-exact).
set -o pipefail
bash tools/ab_envp.sh 2 tum - ORBX_PZ_TILE=96x96 ORBX_PZ_TILE=128x64 ORBX_PZ_TILE=64x96 ORBX_PZ_TILE=160x96
