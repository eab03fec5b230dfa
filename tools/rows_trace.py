"""Per-call breakdown of a tools/prof_rows.sh kernel + memory-copy trace: the drop-in
calls' GPU events (kernels and copies) grouped into calls (a gap of more than GAP_US on
the GPU between two events starts a new call), then per row group the median duration of
each event and of the call's GPU span.
usage: python tools/rows_trace.py TAG  ->  profiles/TAG_rows_call_trace.txt
Calls with the same launch signature (kernel names and grid sizes) in a row form a group.
"""
import csv
import glob
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
GAP_US = 40.0


def events(tag):
    ev = []
    base = ROOT / "gpurun_out" / f"{tag}_rows_prof"
    for p in glob.glob(str(base / "**" / "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("orbx::", "")
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, int(r.get("Grid_Size_X", 0))))
    for p in glob.glob(str(base / "**" / "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            kind = r.get("Direction", r.get("Operation", "copy"))
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), f"copy {kind}", 0))
    ev.sort()
    return ev


def calls(ev):
    """Events grouped into calls: a call starts at the first kernel of an extraction (a
    k_pyramid launch not preceded by another) or, for the matcher rows, after a gap of
    more than GAP_US on the GPU; copies stay with the call they follow."""
    out, cur, last_end, prev = [], [], 0, ""
    for e in ev:
        starts = e[2].startswith("k_pyramid") and not prev.startswith("k_pyramid")
        gap = cur and e[0] - last_end > GAP_US * 1e3 and not e[2].startswith("copy")
        if cur and (starts or (gap and not any(x[2].startswith("k_pyramid") for x in cur))):
            out.append(cur)
            cur = []
        cur.append(e)
        last_end = max(last_end, e[1]) if len(cur) > 1 else e[1]
        prev = e[2]
    if cur:
        out.append(cur)
    return out


def main():
    tag = sys.argv[1]
    cs = [c for c in calls(events(tag)) if any(e[2].startswith("k_") for e in c)]
    lines = [f"# {tag}: drop-in calls under rocprofv3 --kernel-trace --memory-copy-trace (bench.py --rows), "
             f"{len(cs)} calls; per group of consecutive calls with one launch signature (its first call dropped), "
             f"the median us of each event in call order, then of the GPU span (first event start to last event end)"]
    # groups: consecutive calls with the same launch signature (kernel names and grid sizes)
    groups = []
    for c in cs:
        sig = tuple((e[2], e[3]) for e in c if e[2].startswith("k_"))
        if groups and groups[-1][0] == sig:
            groups[-1][1].append(c)
        else:
            groups.append((sig, [c]))
    groups = [(s_, g_) for s_, g_ in groups if len(g_) >= 3]
    for gi, (_, calls_) in enumerate(groups):
        grp = calls_[1:]  # drop the first call of a group (warm-up)
        n = min(len(c) for c in grp)
        cols = []
        for i in range(n):
            name = grp[0][i][2]
            cols.append(f"{name} {statistics.median((c[i][1] - c[i][0]) / 1e3 for c in grp):.1f}")
        span = statistics.median((max(e[1] for e in c) - c[0][0]) / 1e3 for c in grp)
        gaps = statistics.median(((max(e[1] for e in c) - c[0][0]) - sum(e[1] - e[0] for e in c)) / 1e3 for c in grp)
        lines.append(f"group {gi} ({len(grp)} calls): " + " | ".join(cols) +
                     f" | span {span:.1f} (idle between events {gaps:.1f})")
    out = ROOT / "profiles" / f"{tag}_rows_call_trace.txt"
    out.write_text("\n".join(lines) + "\n")
    print("\n".join(lines))
    print("->", out)


if __name__ == "__main__":
    main()
