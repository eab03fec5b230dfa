"""Per-call breakdown of a tools/prof_rows.sh kernel + memory-copy trace: the drop-in
calls' GPU events (kernels and copies) grouped into calls (a gap of more than GAP_US on
the GPU between two events starts a new call), then per row group the median duration of
each event and of the call's GPU span.
usage: python tools/rows_trace.py TAG [CALLS_PER_GROUP]  ->  profiles/TAG_rows_call_trace.txt
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
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    for p in glob.glob(str(base / "**" / "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            kind = r.get("Direction", r.get("Operation", "copy"))
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), f"copy {kind} {r.get('Bytes', '')}B"))
    ev.sort()
    return ev


def calls(ev):
    out, cur, last_end = [], [], 0
    for e in ev:
        if cur and e[0] - last_end > GAP_US * 1e3:
            out.append(cur)
            cur = []
        cur.append(e)
        last_end = max(last_end, e[1]) if len(cur) > 1 else e[1]
    if cur:
        out.append(cur)
    return out


def main():
    tag = sys.argv[1]
    per = int(sys.argv[2]) if len(sys.argv) > 2 else 31
    cs = calls(events(tag))
    lines = [f"# {tag}: drop-in calls under rocprofv3 --kernel-trace --memory-copy-trace (bench.py --rows), "
             f"{len(cs)} calls; per group of {per} consecutive calls (warm-up first), the median us of each "
             f"event in call order, then of the GPU span (first event start to last event end)"]
    for g in range(0, len(cs), per):
        grp = cs[g + 1:g + per] if len(cs[g:g + per]) > 1 else cs[g:g + per]  # drop the warm-up call
        if not grp:
            continue
        n = min(len(c) for c in grp)
        cols = []
        for i in range(n):
            name = grp[0][i][2]
            cols.append(f"{name} {statistics.median((c[i][1] - c[i][0]) / 1e3 for c in grp):.1f}")
        span = statistics.median((max(e[1] for e in c) - c[0][0]) / 1e3 for c in grp)
        gaps = statistics.median(((max(e[1] for e in c) - c[0][0]) - sum(e[1] - e[0] for e in c)) / 1e3 for c in grp)
        lines.append(f"group {g // per}: " + " | ".join(cols) + f" | span {span:.1f} (idle between events {gaps:.1f})")
    out = ROOT / "profiles" / f"{tag}_rows_call_trace.txt"
    out.write_text("\n".join(lines) + "\n")
    print("\n".join(lines))
    print("->", out)


if __name__ == "__main__":
    main()
