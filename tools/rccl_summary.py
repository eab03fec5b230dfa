"""Summarise tools/rccl_ab.sh: the interleaved EuRoC bench lines -- in place, the RCCL
exchange waited for by the matcher stream ("sync", round 4's order) and waited for by the
triangulation stream only ("collective", the default) -- and, from the kernel trace of a
--collective run, what the exchange runs as on the GPU.  At world size 1 RCCL's
all_gather_into_tensor of one rank is a device-to-device copy of the slab (a
__amd_rocclr_copyBuffer launch on the communicator's queue), no RCCL kernel.
usage: python tools/rccl_summary.py TAG [SLAB_MB]  ->  profiles/TAG_rccl_ab.json
"""
import csv
import glob
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
MODES = ("inplace", "sync", "collective")


def main():
    tag = sys.argv[1]
    slab_mb = float(sys.argv[2]) if len(sys.argv) > 2 else 6.1
    base = ROOT / "gpurun_out"
    runs = {m: [] for m in MODES}
    i = 1
    while (base / f"{tag}_euroc_inplace_{i}.json").exists():
        for m in MODES:
            f = base / f"{tag}_euroc_{m}_{i}.json"
            if f.exists():
                d = json.loads(f.read_text().splitlines()[-1])
                runs[m].append({"value": d["value"], "ms_per_step": d["ms_per_step"],
                                "slab_exchange": d["config"].get("slab_exchange")})
        i += 1
    med = {m: statistics.median(r["ms_per_step"] for r in v) for m, v in runs.items() if v}
    copies = []
    for p in glob.glob(str(base / f"{tag}_rccl_prof" / "**" / "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"]
            if "copyBuffer" in name and int(r.get("Grid_Size_X", 0)) >= 65536:  # the slab-sized copies
                copies.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            if any(t in name.lower() for t in ("nccl", "rccl")):
                copies.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {"what": "configs[3] EuRoC step: the RCCL all_gather_into_tensor of the keyframe slabs at world size 1 "
                   "(bench.py --workload euroc --collective) against the in-place step, interleaved on one box",
           "runs": runs, "ms_per_step_median": med,
           "step_ms_added_sync": round(med["sync"] - med["inplace"], 4) if "sync" in med else None,
           "step_ms_added_async": round(med["collective"] - med["inplace"], 4) if "collective" in med else None,
           "exchange_on_gpu": {"launches": len(copies),
                               "duration_us_median": round(statistics.median(copies), 1) if copies else None,
                               "note": "world size 1: RCCL's one-rank all-gather is a device copy of the slab"},
           "slab_mb": slab_mb}
    dst = ROOT / "profiles" / f"{tag}_rccl_ab.json"
    dst.write_text(json.dumps(out, indent=1))
    print(json.dumps({k: out[k] for k in ("ms_per_step_median", "step_ms_added_sync", "step_ms_added_async",
                                          "exchange_on_gpu")}, indent=1))
    print("->", dst)


if __name__ == "__main__":
    main()
