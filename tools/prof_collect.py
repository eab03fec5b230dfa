"""Copy one workload's profile summaries from gpurun_out/ (tools/prof_bench.sh) into
profiles/: <TAG>_<WL>_kernel_stats.csv (rocprofv3 --stats), <TAG>_<WL>_pmc_traffic.json
(tools/pmc_traffic.py's per-launch HBM bytes) and <TAG>_<WL>_prof_bench.json (the bench
line of the profiled run, whose HIP-event times sit beside the trace's), and
<TAG>_<WL>_kernel_stats_timed.csv: the same statistics over the launches of the bench's
timed steps only (the later legs -- TrackLocalMap, host-fed -- run the kernels beside
other work, so the whole trace's means are not the timed region's).
usage: python tools/prof_collect.py TAG WORKLOAD [STEPS]"""
import csv
import glob
import math
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def timed_stats(trace_csv: str, steps: int, out: Path, lanes: int = 2, gap_ms: float = 5.0) -> None:
    """Per-kernel statistics over the timed steps of the bench's first leg: every step
    launches k_pyramid `lanes` x segments times (two lanes, or the left and right
    extractors; one launch per pyramid segment); that
    leg ends at the first pause of more than gap_ms between pyramid launches after its
    last launches could have begun (or at the trace's end), and its timed steps are its
    last lanes * segments * steps pyramid launches.  Kernels that start from the first of
    them up to the next leg's first pyramid launch are counted."""
    ev = []
    for r in csv.DictReader(open(trace_csv)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ev.sort()
    def is_(e, k):
        return e[2].split("(")[0].replace("void ", "").startswith(k)
    pyr = [e for e in ev if is_(e, "orbx::k_pyramid")]
    # a deep pyramid is built in segments, one k_pyramid launch each (configs[4]'s 12
    # levels: 2): launches per extraction = k_pyramid / k_level_tiles launches (one each)
    nlt = sum(1 for e in ev if is_(e, "orbx::k_level_tiles"))
    nseg = max(1, round(len(pyr) / nlt)) if nlt else 1
    n = lanes * nseg * steps
    if len(pyr) < n:
        return
    end = len(pyr) - 1
    for i in range(n - 1, len(pyr) - 1):
        if (pyr[i + 1][0] - pyr[i][0]) / 1e6 > gap_ms:
            end = i
            break
    t0 = pyr[end - n + 1][0]
    t1 = pyr[end + 1][0] if end + 1 < len(pyr) else math.inf
    per = {}
    for s_, e_, name in ev:
        if t0 <= s_ < t1:
            per.setdefault(name, []).append(e_ - s_)
    tot = sum(sum(v) for v in per.values()) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for name, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
            m = sum(d) / len(d)
            sd = math.sqrt(sum((x - m) ** 2 for x in d) / len(d))
            w.writerow([name, len(d), sum(d), m, 100.0 * sum(d) / tot, min(d), max(d), sd])


def main():
    tag, wl = sys.argv[1], sys.argv[2]
    base = ROOT / "gpurun_out"
    stats = glob.glob(str(base / f"{tag}_{wl}_prof" / "**" / "*kernel_stats.csv"), recursive=True)
    if not stats:
        raise SystemExit("no kernel_stats.csv")
    shutil.copy(stats[0], ROOT / "profiles" / f"{tag}_{wl}_kernel_stats.csv")
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    trace = glob.glob(str(base / f"{tag}_{wl}_prof" / "**" / "*kernel_trace.csv"), recursive=True)
    if trace:
        timed_stats(trace[0], steps, ROOT / "profiles" / f"{tag}_{wl}_kernel_stats_timed.csv")
    line = (base / f"{tag}_{wl}_prof.json").read_text().strip().splitlines()[-1]
    (ROOT / "profiles" / f"{tag}_{wl}_prof_bench.json").write_text(line + "\n")
    # tools/pmc_traffic.py reads gpurun_out/<T>_fetch and <T>_write for T = f"{tag}_{wl}"
    subprocess.run([sys.executable, str(ROOT / "tools" / "pmc_traffic.py"), f"{tag}_{wl}"], check=True)
    print("collected", tag, wl)


if __name__ == "__main__":
    main()
