"""Copy one workload's profile summaries from gpurun_out/ (tools/prof_bench.sh) into
profiles/: <TAG>_<WL>_kernel_stats.csv (rocprofv3 --stats), <TAG>_<WL>_pmc_traffic.json
(tools/pmc_traffic.py's per-launch HBM bytes) and <TAG>_<WL>_prof_bench.json (the bench
line of the profiled run, whose HIP-event times sit beside the trace's).
usage: python tools/prof_collect.py TAG WORKLOAD"""
import glob
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def main():
    tag, wl = sys.argv[1], sys.argv[2]
    base = ROOT / "gpurun_out"
    stats = glob.glob(str(base / f"{tag}_{wl}_prof" / "**" / "*kernel_stats.csv"), recursive=True)
    if not stats:
        raise SystemExit("no kernel_stats.csv")
    shutil.copy(stats[0], ROOT / "profiles" / f"{tag}_{wl}_kernel_stats.csv")
    line = (base / f"{tag}_{wl}_prof.json").read_text().strip().splitlines()[-1]
    (ROOT / "profiles" / f"{tag}_{wl}_prof_bench.json").write_text(line + "\n")
    # tools/pmc_traffic.py reads gpurun_out/<T>_fetch and <T>_write for T = f"{tag}_{wl}"
    subprocess.run([sys.executable, str(ROOT / "tools" / "pmc_traffic.py"), f"{tag}_{wl}"], check=True)
    print("collected", tag, wl)


if __name__ == "__main__":
    main()
