"""Host-side measurement logic of bench.py (no GPU): the algorithmic bytes per frame are
SURVEY.md §8(d)'s canonical figures, level sizes follow ORBextractor.cc:1641-1643, and
the PMC summaries under profiles/ resolve to every extraction stage's kernels."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def test_level_sizes_c1():
    # SURVEY.md §8 table, C1
    assert bench.level_areas(640, 480) == [(640, 480), (533, 400), (444, 333), (370, 278), (309, 231),
                                           (257, 193), (214, 161), (179, 134)]


def test_b_frame_matches_survey():
    # C1, C3 (per image), C5
    assert bench.stage_bytes(640, 480, 1000)["total"] == 3_862_128
    assert bench.stage_bytes(1241, 376, 2000)["total"] == 5_896_388
    assert bench.stage_bytes(640, 480, 5000, nlevels=12)["total"] == 4_269_504


def test_score_blur_bytes_are_three_passes():
    P = sum(w * h for w, h in bench.level_areas(640, 480))
    assert P == 950_532
    assert bench.stage_bytes(640, 480, 1000)["score_blur"] == 3 * P


def test_pmc_summaries_cover_the_stages():
    for stage in ("pyramid", "score_blur", "fast_cells", "octree", "describe", "match"):
        t, src = bench.pmc_traffic(stage)
        v, vsrc = bench.pmc_valu(stage)
        assert t is not None and t > 0, (stage, src)
        assert v is not None and v > 0, (stage, vsrc)


def test_stage_sum_prefix_and_missing():
    ks = {"orbx::k_seq_build": {"x": 1}, "orbx::k_proj_search<false, false, 1024, true>": {"x": 2},
          "orbx::k_seq_commit": {"x": 4}}
    assert bench._stage_sum(ks, "match", "x") == 7
    assert bench._stage_sum({k: v for k, v in ks.items() if "commit" not in k}, "match", "x") is None
    assert bench._stage_sum(ks, "pyramid", "x") is None
    assert bench._stage_sum({}, "no-such-stage", "x") is None


def test_profile_fields_read_the_workload_trace(tmp_path, monkeypatch):
    """A bench line's rocprof mean comes from the newest <tag>_<workload>_kernel_stats.csv and
    its frac_rocprof follows from it and the algorithmic bytes."""
    prof = tmp_path / "profiles"
    prof.mkdir()
    hdr = '"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n'
    (prof / "r03a_tum_kernel_stats.csv").write_text(
        hdr + '"orbx::k_level_tiles(unsigned char const*)",50,1,400000.0,1,1,1,1\n')
    (prof / "r03b_tum_kernel_stats.csv").write_text(
        hdr + '"orbx::k_level_tiles(unsigned char const*)",50,1,300000.0,1,1,1,1\n')
    (prof / "r03c_tum5k_kernel_stats.csv").write_text(
        hdr + '"orbx::k_level_tiles(unsigned char const*)",50,1,900000.0,1,1,1,1\n')
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    f = bench.profile_fields("score_blur", 2.4e8, 0.3, "tum")
    assert f["rocprof_source"] == "r03b_tum_kernel_stats.csv" and f["rocprof_mean_ms"] == 0.3
    assert abs(f["frac_rocprof"] - 2.4e8 / 0.3e-3 / 1e9 / bench.HBM_PEAK_GBS) < 1e-5
    assert bench.profile_fields("score_blur", 1.0, 0.3, "kitti")["rocprof_mean_ms"] is None


def test_dominant_stage_prefers_the_kernel_trace(tmp_path, monkeypatch):
    """Pipelined HIP-event times hold queueing beside the other streams, so the roofline's
    kernel is the longest one in the workload's kernel trace when that covers every stage
    (here describe's events are longest but its kernel is not), and the events decide
    otherwise."""
    prof = tmp_path / "profiles"
    prof.mkdir()
    hdr = '"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n'
    (prof / "r03e_tum_kernel_stats.csv").write_text(
        hdr + '"orbx::k_level_tiles(unsigned char const*)",50,1,316000.0,1,1,1,1\n'
        '"void orbx::k_describe<true>(unsigned char const*)",50,1,263000.0,1,1,1,1\n')
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    ev = {"score_blur": 0.314, "describe": 0.313}
    ev2 = {"score_blur": 0.30, "describe": 0.31}
    assert bench.dominant_stage(ev2, "tum") == "score_blur"
    assert bench.dominant_stage(ev, "kitti") == "score_blur"  # no trace: events
    assert bench.dominant_stage({**ev2, "pyramid": 0.1}, "tum") == "describe"  # pyramid not in the trace


def test_newest_profile_is_highest_tag():
    files = bench.newest_profiles("*_pmc_traffic.json")
    assert files, "no PMC traffic summary under profiles/"
    data = json.loads(files[-1].read_text())
    assert "orbx::k_level_tiles" in data["kernels"]


def test_newest_profiles_prefer_the_current_source(tmp_path, monkeypatch):
    """A pass taken at the code's current source hash counts as newest whatever its tag's
    letter; without one, the tags' numbers and names decide."""
    prof = tmp_path / "profiles"
    prof.mkdir()
    for tag, h in (("r04n", "old"), ("r04f", "cur")):
        (prof / f"{tag}_tum_pmc_traffic.json").write_text(json.dumps({"source_hash": h, "kernels": {}}))
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    monkeypatch.setattr(bench, "_SRC_HASH", "cur")
    assert [f.name for f in bench.newest_profiles("*_pmc_traffic.json")][-1] == "r04f_tum_pmc_traffic.json"
    monkeypatch.setattr(bench, "_SRC_HASH", "other")
    assert [f.name for f in bench.newest_profiles("*_pmc_traffic.json")][-1] == "r04n_tum_pmc_traffic.json"


def test_gpus_flag_launches_that_many_ranks():
    """bench.py --gpus 2 with no launcher starts two ranks itself (the path the driver's
    N>1 runs take when WORLD_SIZE is unset); each joins the group (gloo here)."""
    import subprocess
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--selftest-launch"],
                       capture_output=True, text=True, timeout=240, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout
    out = json.loads(line[0])
    assert out["world"] == 2 and out["gpus"] == 2 and out["rank_sum"] == 3


def test_gpus_flag_must_match_world_size():
    import os
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--selftest-launch"],
                       capture_output=True, text=True, timeout=120, env=env, cwd="/tmp")
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def test_cpu_baseline_build_matches_checker(oracle):
    """The -O3 -march=native baseline build reproduces the -O2 checker bit for bit."""
    import numpy as np
    from orbslam2commentedbyxcm_amd import synth
    frames = synth.frames(2, first_seed=40)
    p = oracle.params()
    ref = [oracle.extract(f, p) for f in frames]
    flags = oracle.select("native")
    try:
        nat = [oracle.extract(f, p) for f in frames]
    finally:
        oracle.select("parity")
    assert "-O3" in flags
    for (k0, d0, _), (k1, d1, _) in zip(ref, nat):
        assert np.array_equal(k0.view(np.uint8), k1.view(np.uint8)) and np.array_equal(d0, d1)


def test_h3_flip_count_runs(oracle):
    """cosf/sinf (the reference's literal H3 arithmetic) vs the shipped correctly rounded
    cos/sin: same keypoints; the descriptor difference is counted (profiles/r02_h3_flips.json
    holds the 256-frame figure)."""
    sys.path.insert(0, str(ROOT / "benchmarks"))
    import h3_flip_count
    from orbslam2commentedbyxcm_amd import synth
    r = h3_flip_count.count_flips(synth.frames(3, first_seed=90), threads=3)
    assert r["keypoints_identical_all_frames"] and r["keypoints"] > 2000
    assert r["descriptors_differing"] <= r["keypoints"] // 100


def test_rocprof_mean_prefers_the_timed_steps(tmp_path, monkeypatch):
    """tools/prof_collect.py's statistics over the timed steps' launches win over the
    whole trace's (whose later legs run the kernels beside other work)."""
    prof = tmp_path / "profiles"
    prof.mkdir()
    hdr = '"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n'
    (prof / "r03g_tum5k_kernel_stats.csv").write_text(hdr + '"orbx::k_pyramid<true>(x)",150,1,408000.0,1,1,1,1\n')
    (prof / "r03g_tum5k_kernel_stats_timed.csv").write_text(hdr + '"orbx::k_pyramid<true>(x)",40,1,587000.0,1,1,1,1\n')
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    ms, src = bench.rocprof_mean_ms("pyramid", "tum5k")
    assert src == "r03g_tum5k_kernel_stats_timed.csv" and abs(ms - 0.587) < 1e-9


def test_prof_collect_timed_window(tmp_path):
    """The timed steps are the first leg's last lanes x steps pyramid launches; kernels
    from the first of them up to the next leg's first pyramid launch are counted."""
    import csv
    import importlib.util
    spec = importlib.util.spec_from_file_location("prof_collect", ROOT / "tools" / "prof_collect.py")
    pc = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(pc)
    rows, t = [], 0
    def add(name, dur):
        nonlocal t
        rows.append({"Start_Timestamp": t, "End_Timestamp": t + dur, "Kernel_Name": name})
        t += dur
    for step in range(6):          # leg 1: 2 warmup + 4 timed steps, 2 lanes
        for lane in range(2):
            add("void orbx::k_pyramid<true>(a)", 100 if step >= 2 else 999)
            add("orbx::k_describe(a)", 50)
    t += 50_000_000                # the next leg starts 50 ms later
    for step in range(3):
        add("void orbx::k_pyramid<true>(a)", 7777)
    trace = tmp_path / "trace.csv"
    with open(trace, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Start_Timestamp", "End_Timestamp", "Kernel_Name"])
        w.writeheader()
        w.writerows(rows)
    out = tmp_path / "timed.csv"
    pc.timed_stats(str(trace), 4, out)
    got = {r["Name"]: (int(r["Calls"]), float(r["AverageNs"])) for r in csv.DictReader(open(out))}
    assert got["void orbx::k_pyramid<true>(a)"] == (8, 100.0)
    assert got["orbx::k_describe(a)"] == (8, 50.0)


def test_prof_collect_timed_window_pyramid_segments(tmp_path):
    """A 12-level pyramid is two k_pyramid launches per extraction (one per segment): the
    timed window still spans the last `steps` steps, found from the k_pyramid /
    k_level_tiles launch ratio."""
    import csv
    import importlib.util
    spec = importlib.util.spec_from_file_location("prof_collect", ROOT / "tools" / "prof_collect.py")
    pc = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(pc)
    rows, t = [], 0

    def add(name, dur):
        nonlocal t
        rows.append({"Start_Timestamp": t, "End_Timestamp": t + dur, "Kernel_Name": name})
        t += dur
    for step in range(6):          # 2 warmup + 4 timed steps, 2 lanes, 2 segments
        for lane in range(2):
            add("void orbx::k_pyramid<true>(a)", 100 if step >= 2 else 999)
            add("void orbx::k_pyramid<true>(a)", 20 if step >= 2 else 999)
            add("orbx::k_level_tiles(a)", 70 if step >= 2 else 999)
    trace = tmp_path / "trace.csv"
    with open(trace, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Start_Timestamp", "End_Timestamp", "Kernel_Name"])
        w.writeheader()
        w.writerows(rows)
    out = tmp_path / "timed.csv"
    pc.timed_stats(str(trace), 4, out)
    got = {r["Name"]: (int(r["Calls"]), float(r["AverageNs"])) for r in csv.DictReader(open(out))}
    assert got["void orbx::k_pyramid<true>(a)"] == (16, 60.0)
    assert got["orbx::k_level_tiles(a)"] == (8, 70.0)


def test_stage_sum_counts_pyramid_segments(tmp_path, monkeypatch):
    """The pyramid stage per extraction is k_pyramid's mean launch x its launches per
    extraction (k_pyramid calls / k_level_tiles calls), in the trace and PMC summaries."""
    prof = tmp_path / "profiles"
    prof.mkdir()
    hdr = '"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n'
    (prof / "r09_tum5k_kernel_stats_timed.csv").write_text(
        hdr + '"void orbx::k_pyramid<true>(x)",80,1,300000.0,1,1,1,1\n"orbx::k_level_tiles(x)",40,1,1,1,1,1,1\n')
    (prof / "r09_tum5k_pmc_traffic.json").write_text(json.dumps({"kernels": {
        "orbx::k_pyramid<true>": {"traffic_bytes": 1000, "dispatches": 6},
        "orbx::k_level_tiles": {"traffic_bytes": 5, "dispatches": 3}}}))
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    ms, _ = bench.rocprof_mean_ms("pyramid", "tum5k")
    assert abs(ms - 0.6) < 1e-9
    assert bench.pmc_traffic("pyramid", "tum5k")[0] == 2000
    assert bench.pmc_traffic("score_blur", "tum5k")[0] == 5


def test_pmc_valu_reads_the_workload_file(tmp_path, monkeypatch):
    """The issue figure comes from the newest VALU summary of the bench's own workload
    (configs[1]: <tag>_tum_ or untagged files, never another workload's), and a summary
    taken at other sources than the running code is flagged stale."""
    import json
    prof = tmp_path / "profiles"
    prof.mkdir()

    def put(name, valu, h):
        (prof / name).write_text(json.dumps({"source_hash": h, "kernels": {
            "orbx::k_level_tiles": {"sq_insts_valu": valu, "dispatches": 4}}}))
    put("r03c_pmc_valu.json", 100, "x")
    put("r04a_tum5k_pmc_valu.json", 900, "y")
    put("r04a_tum_pmc_valu.json", 200, bench.source_hash())
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    assert bench.pmc_valu("score_blur", "tum") == (200, "r04a_tum_pmc_valu.json")
    assert bench.pmc_valu("score_blur", "tum5k") == (900, "r04a_tum5k_pmc_valu.json")
    assert bench.pmc_valu("score_blur", "kitti") == (None, None)
    assert bench.profile_hash(prof / "r04a_tum_pmc_valu.json") == bench.source_hash()
    assert bench.profile_hash(prof / "r04a_tum5k_pmc_valu.json") != bench.source_hash()


def test_source_hash_tracks_the_sources():
    h = bench.source_hash()
    assert len(h) == 16 and h == bench.source_hash()


def test_exchange_leg_arguments():
    # the N-GPU headline's keyframe-exchange leg: euroc_bench.parse / run as bench.py calls them
    sys.path.insert(0, str(ROOT / "benchmarks"))
    import inspect

    import euroc_bench
    a = euroc_bench.parse(["--steps", "10", "--warmup", "3", "--no-cpu-baseline"])
    assert (a.steps, a.warmup, a.batch, a.nn, a.no_cpu_baseline, a.parity_frames) == (10, 3, 64, 10, True, -1)
    assert list(inspect.signature(euroc_bench.run).parameters) == ["args", "rank", "world", "device", "collective"]
    src = (ROOT / "bench.py").read_text()
    assert '"--no-exchange"' in src and "euroc_bench.run(eargs, rank, world, gpu, True)" in src
    assert '"keyframe_exchange": exchange' in src
