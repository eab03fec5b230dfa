"""Summarise FETCH_SIZE / WRITE_SIZE passes (tools/pmc_traffic.sh) into per-launch HBM
bytes per kernel.

rocprofv3 reports FETCH_SIZE and WRITE_SIZE in KiB per dispatch.  On gfx950 FETCH_SIZE
counts 64 B per 128-B read request, i.e. half the bytes of wide streaming reads
(MI355X_MICROARCH.md "HBM"), so reads are doubled; WRITE_SIZE is taken as is.
usage: python tools/pmc_traffic.py TAG  ->  profiles/TAG_pmc_traffic.json
"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def per_kernel(pattern, counter):
    acc = defaultdict(list)
    for p in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            acc[(name, r.get("Dispatch_Id", r.get("Correlation_Id", "")))].append(float(r["Counter_Value"]))
    out = defaultdict(list)
    for (name, _), vals in acc.items():
        out[name].append(sum(vals))  # sum over XCD / instance rows of one dispatch
    return {k: sum(v) / len(v) for k, v in out.items()}, {k: len(v) for k, v in out.items()}


def bench_source_hash(*logs):
    """The source_hash of the bench line a profiled run printed (its last JSON line)."""
    for log in logs:
        try:
            for line in reversed(Path(log).read_text().splitlines()):
                if line.startswith("{"):
                    return json.loads(line).get("source_hash")
        except (OSError, ValueError):
            continue
    return None


def main():
    tag = sys.argv[1]
    base = ROOT / "gpurun_out"
    fetch, nf = per_kernel(str(base / f"{tag}_fetch" / "**" / "*counter_collection.csv"), "FETCH_SIZE")
    write, nw = per_kernel(str(base / f"{tag}_write" / "**" / "*counter_collection.csv"), "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        rd = 2.0 * fetch.get(k, 0.0) * 1024.0
        wr = write.get(k, 0.0) * 1024.0
        res[k] = {"read_bytes": round(rd), "write_bytes": round(wr), "traffic_bytes": round(rd + wr),
                  "dispatches": nf.get(k, 0)}
    out = ROOT / "profiles" / f"{tag}_pmc_traffic.json"
    out.write_text(json.dumps({"units": "bytes per launch (FETCH_SIZE x2 x1024 + WRITE_SIZE x1024)",
                               "source_hash": bench_source_hash(base / f"{tag}_fetch.log", base / f"{tag}_write.log"),
                               "kernels": res}, indent=1))
    for k, v in res.items():
        print(f"{k:40s} read {v['read_bytes']/1e6:10.2f} MB  write {v['write_bytes']/1e6:10.2f} MB  "
              f"n={v['dispatches']}")
    print("->", out)


if __name__ == "__main__":
    main()
