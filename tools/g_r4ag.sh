# configs[4] describe staging: register (base) vs LDS-DMA 4-byte (dma) and 16-byte (dma1),
# now that the matcher beside it is lighter; interleaved pipelined A/B.
set -o pipefail
STEPS=20 bash tools/ab_lib.sh 3 tum5k base dma dma1 || exit 1
echo ok
