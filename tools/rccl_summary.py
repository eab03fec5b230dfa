"""Summarise tools/rccl_ab.sh: the interleaved in-place / --collective EuRoC bench lines
(rate and step time per pair, the difference) and, from the kernel trace of the
--collective run, the RCCL kernels' durations and the idle time they leave on their queue
(from the end of the kernel before each collective to the start of the kernel after it).
usage: python tools/rccl_summary.py TAG  ->  profiles/TAG_rccl_ab.json
"""
import csv
import glob
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def main():
    tag = sys.argv[1]
    base = ROOT / "gpurun_out"
    pairs = []
    i = 1
    while (base / f"{tag}_euroc_inplace_{i}.json").exists():
        row = {}
        for mode in ("inplace", "collective"):
            d = json.loads((base / f"{tag}_euroc_{mode}_{i}.json").read_text().splitlines()[-1])
            row[mode] = {"value": d["value"], "ms_per_step": d["ms_per_step"],
                         "slab_exchange": d["config"].get("slab_exchange")}
        row["step_ms_added"] = round(row["collective"]["ms_per_step"] - row["inplace"]["ms_per_step"], 4)
        pairs.append(row)
        i += 1
    ev = []
    for p in glob.glob(str(base / f"{tag}_rccl_prof" / "**" / "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
                       r.get("Queue_Id", r.get("Stream_Id"))))
    ev.sort()
    coll = [k for k, e in enumerate(ev) if any(t in e[2].lower() for t in ("nccl", "rccl"))]
    durs, gaps = [], []
    for k in coll:
        s, e, _, q = ev[k]
        durs.append((e - s) / 1e3)
        prev = [x for x in ev[:k] if x[3] == q]
        nxt = [x for x in ev[k + 1:] if x[3] == q]
        if prev and nxt:
            gaps.append((nxt[0][0] - prev[-1][1]) / 1e3)
    out = {"what": "configs[3] EuRoC step with the RCCL all_gather_into_tensor of the keyframe slabs (world size 1: "
                   "a self-gather through the process group) against the in-place step, interleaved on one box",
           "pairs": pairs,
           "step_ms_added_median": statistics.median(p["step_ms_added"] for p in pairs) if pairs else None,
           "step_ms_inplace_median": statistics.median(p["inplace"]["ms_per_step"] for p in pairs) if pairs else None,
           "rccl_kernels": {"launches": len(durs), "names": sorted({ev[k][2] for k in coll}),
                            "duration_us_median": round(statistics.median(durs), 2) if durs else None,
                            "queue_span_us_median": round(statistics.median(gaps), 2) if gaps else None,
                            "note": "queue span: end of the kernel before the collective to the start of the kernel "
                                    "after it on the same queue"}}
    dst = ROOT / "profiles" / f"{tag}_rccl_ab.json"
    dst.write_text(json.dumps(out, indent=1))
    print(json.dumps(out, indent=1))
    print("->", dst)


if __name__ == "__main__":
    main()
