"""Summarise a tools/pmc_valu.sh pass into per-launch vector-issue figures per kernel.

SQ_INSTS_VALU counts wave-instructions.  A SIMD issues one wave64 VALU instruction per
2 cycles (MI355X_MICROARCH.md, "Wave scheduling"), so the chip's issue ceiling is
1024 SIMDs x 2.4 GHz / 2 = 1.2288e12 wave-instructions/s; bench.py divides a stage's
VALU count per launch by its measured time to place it under that ceiling.
usage: python tools/pmc_valu.py TAG_WORKLOAD  ->  profiles/TAG_WORKLOAD_pmc_valu.json
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import ROOT, bench_source_hash, per_kernel  # noqa: E402


def main():
    tag = sys.argv[1]
    pat = str(ROOT / "gpurun_out" / f"{tag}_valu" / "**" / "*counter_collection.csv")
    res = {}
    cols = {c: per_kernel(pat, c) for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES")}
    names = set()
    for v, _ in cols.values():
        names |= set(v)
    for k in sorted(names):
        res[k] = {c.lower(): round(cols[c][0].get(k, 0.0)) for c in cols}
        res[k]["dispatches"] = cols["SQ_INSTS_VALU"][1].get(k, 0)
    out = ROOT / "profiles" / f"{tag}_pmc_valu.json"
    out.write_text(json.dumps({"units": "wave-instructions (and waves) per launch",
                               "valu_issue_peak_per_s": 1024 * 2.4e9 / 2,
                               "source_hash": bench_source_hash(ROOT / "gpurun_out" / f"{tag}_valu.log"),
                               "kernels": res}, indent=1))
    for k, v in res.items():
        print(f"{k:40s} valu {v['sq_insts_valu']/1e6:8.2f} M  lds {v['sq_insts_lds']/1e6:7.2f} M  waves {v['sq_waves']}")
    print("->", out)


if __name__ == "__main__":
    main()
