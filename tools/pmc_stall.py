"""Summarise a tools/pmc_stall.sh pass: per kernel launch, the wave-cycle split
(ACTIVE_INST_ANY + WAIT_INST_ANY + WAIT_ANY ~= WAVE_CYCLES, MI355X_MICROARCH.md PMC
table; all in quad-cycles) and the LDS array's busy / bank-conflict cycles.
usage: python tools/pmc_stall.py TAG  ->  profiles/TAG_pmc_stall.json
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import ROOT, per_kernel  # noqa: E402

COUNTERS = ("SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU",
            "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS")


def main():
    tag = sys.argv[1]
    pat = str(ROOT / "gpurun_out" / f"{tag}_stall" / "**" / "*counter_collection.csv")
    cols = {c: per_kernel(pat, c)[0] for c in COUNTERS}
    res = {}
    for k in sorted(cols["SQ_WAVE_CYCLES"]):
        if not k.startswith("orbx::"):
            continue
        v = {c.lower(): round(cols[c].get(k, 0.0)) for c in COUNTERS}
        wc = max(v["sq_wave_cycles"], 1)
        v["frac_active"] = round(v["sq_active_inst_any"] / wc, 3)
        v["frac_issue_stall"] = round(v["sq_wait_inst_any"] / wc, 3)
        v["frac_wait"] = round(v["sq_wait_any"] / wc, 3)
        v["lds_conflict_frac"] = round(v["sq_lds_bank_conflict"] / max(v["sq_lds_idx_active"], 1), 3)
        res[k] = v
    out = ROOT / "profiles" / f"{tag}_pmc_stall.json"
    out.write_text(json.dumps({"units": "quad-cycles per launch summed over waves", "kernels": res}, indent=1))
    for k, v in res.items():
        print(f"{k:34s} active {v['frac_active']:.2f} issue-stall {v['frac_issue_stall']:.2f} "
              f"wait {v['frac_wait']:.2f}  lds-conflict {v['lds_conflict_frac']:.2f}")
    print("->", out)


if __name__ == "__main__":
    main()
