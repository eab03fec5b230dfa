"""Summarise a tools/pmc_stall.sh run: per kernel launch, the wave-cycle split
(ACTIVE_INST_ANY + WAIT_INST_ANY + WAIT_ANY ~= WAVE_CYCLES, MI355X_MICROARCH.md PMC
table; SQ cycle counters count quad-cycles), the mean resident waves, VALU issue, the LDS
array's busy / bank-conflict cycles and the effective clock, and names the resource that
bounds each kernel.
usage: python tools/pmc_stall.py TAG [KERNEL_TRACE_STATS_CSV]  ->  profiles/TAG_pmc_stall.json

Occupancy and the issue / LDS fractions need each launch's cycles: GRBM_GUI_ACTIVE / 8
from the same serialised counter run (the kernel alone), else the kernel-trace stats CSV
given (e.g. profiles/<tag>_tum_kernel_stats_timed.csv) at 2.4 GHz.
"""
import csv
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import ROOT, bench_source_hash, per_kernel  # noqa: E402

PASS_A = ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
          "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT")
PASS_B = ("SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS",
          "SQ_INSTS_SALU", "SQ_ACTIVE_INST_SCA", "SQ_INST_CYCLES_VMEM", "GRBM_GUI_ACTIVE")
CUS, SIMDS, CLOCK_GHZ = 256, 1024, 2.4


def trace_durations(path):
    """Mean duration (ns) per kernel from a rocprofv3 kernel_stats CSV."""
    out = {}
    if not path:
        return out
    for r in csv.DictReader(open(path)):
        out[r["Name"].split("(")[0].replace("void ", "")] = float(r["AverageNs"])
    return out


def classify(v):
    """The resource that bounds a kernel, from its counters."""
    if v.get("valu_issue_frac", 0) > 0.6:
        return "VALU issue"
    if v.get("lds_busy_frac", 0) > 0.6:
        return "LDS array"
    if v["frac_wait"] > 0.5:
        return "latency (waitcnt / barrier): memory or LDS round trips not hidden at this occupancy"
    if v["frac_issue_stall"] > 0.35:
        return "issue stalls (dependent instructions, LDS queue)"
    return "mixed"


def main():
    tag = sys.argv[1]
    durs = trace_durations(sys.argv[2] if len(sys.argv) > 2 else None)
    base = ROOT / "gpurun_out"
    cols = {}
    for p, names in (("A", PASS_A), ("B", PASS_B)):
        pat = str(base / f"{tag}_stall{p}" / "**" / "*counter_collection.csv")
        for c in names:
            vals, _ = per_kernel(pat, c)
            if vals:
                cols[c] = vals
    res = {}
    for k in sorted(cols.get("SQ_WAVE_CYCLES", {})):
        if not k.startswith("orbx::"):
            continue
        v = {c.lower(): round(cols[c].get(k, 0.0)) for c in cols}
        wc = max(v["sq_wave_cycles"], 1)
        v["frac_active"] = round(v.get("sq_active_inst_any", 0) / wc, 3)
        v["frac_issue_stall"] = round(v.get("sq_wait_inst_any", 0) / wc, 3)
        v["frac_wait"] = round(v.get("sq_wait_any", 0) / wc, 3)
        if "sq_lds_idx_active" in v:
            v["lds_conflict_frac"] = round(v.get("sq_lds_bank_conflict", 0) / max(v["sq_lds_idx_active"], 1), 3)
        # the launch's shader cycles: GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 -- taken in
        # the same serialised counter run, so it is the kernel alone at whatever clock it ran;
        # else a kernel trace's mean duration at 2.4 GHz
        cyc = v["grbm_gui_active"] / 8 if v.get("grbm_gui_active") else None
        if cyc is None and durs.get(k):
            cyc = durs[k] * CLOCK_GHZ
        if cyc:
            v["launch_cycles"] = round(cyc)
            if durs.get(k):
                v["trace_duration_ns"] = round(durs[k])
            v["mean_waves_per_simd"] = round(4 * wc / cyc / SIMDS, 2)   # wave-cycles are quad-cycles
            if "sq_insts_valu" in v:
                v["valu_issue_frac"] = round(v["sq_insts_valu"] / (cyc * SIMDS / 2), 3)  # one wave64 VALU / 2 cyc / SIMD
            if "sq_lds_idx_active" in v:
                v["lds_busy_frac"] = round(v["sq_lds_idx_active"] / (cyc * CUS), 3)  # LDS-array cycles per CU-cycle
        v["bound"] = classify(v)
        res[k] = v
    out = ROOT / "profiles" / f"{tag}_pmc_stall.json"
    out.write_text(json.dumps({"units": "SQ cycle counters in quad-cycles, per launch, summed over waves",
                               "source_hash": bench_source_hash(base / f"{tag}_stallA.log"),
                               "cycles_from": "GRBM_GUI_ACTIVE / 8 (same counter run, dispatches serialised)",
                               "kernels": res}, indent=1))
    for k, v in res.items():
        print(f"{k:34s} waves/SIMD {v.get('mean_waves_per_simd', '-')} active {v['frac_active']:.2f} "
              f"issue-stall {v['frac_issue_stall']:.2f} wait {v['frac_wait']:.2f} "
              f"valu {v.get('valu_issue_frac', '-')} lds-busy {v.get('lds_busy_frac', '-')} "
              f"lds-conflict {v.get('lds_conflict_frac', '-')} -> {v['bound']}")
    print("->", out)


if __name__ == "__main__":
    main()
