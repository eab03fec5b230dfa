"""Summarise tools/pmc_lanes.sh: per kernel launch, the VALU lane utilisation
(SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)) and instructions per wave.
usage: python tools/pmc_lanes.py TAG
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import ROOT, per_kernel  # noqa: E402

CTRS = ("SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH",
        "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_WAVES")


def main():
    tag = sys.argv[1]
    pat = str(ROOT / "gpurun_out" / f"{tag}_lanes" / "**" / "*counter_collection.csv")
    v = {c: per_kernel(pat, c)[0] for c in CTRS}
    for k in sorted(v["SQ_WAVES"]):
        w = v["SQ_WAVES"][k] or 1
        act = v["SQ_ACTIVE_INST_VALU"].get(k, 0)
        util = v["SQ_THREAD_CYCLES_VALU"].get(k, 0) / (64 * act) if act else 0
        per = {c.replace("SQ_INSTS_", ""): round(v[c].get(k, 0) / w) for c in CTRS[2:7]}
        print(f"{k[:48]:48s} waves {w:8.0f} lane-util {util:.3f} per wave {per}")


if __name__ == "__main__":
    main()
