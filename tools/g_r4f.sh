set -o pipefail
timeout -k 10 300 python tools/timing_ab.py 4 20 5 && timeout -k 10 300 python tools/timing_ab.py 2 100 20
