#!/usr/bin/env python3
"""configs[3] throughput: a frame-sharded EuRoC-shaped stereo keyframe stream with the
cross-keyframe exchange, on 1..8 MI355X (one process per GPU).

    python bench.py --workload euroc [--gpus N] [--steps K] [--warmup W] [--batch B]

(bench.py's configs[3] leg; it runs the oracle as its parity check and CPU baseline;
bench.py --gpus N starts the ranks.)

Workload (orbslam2commentedbyxcm_amd/keyframes.py): per rank and step, B = 64 stereo
keyframes of a window of N*B (keyframe g on rank g % N) -- synthetic rectified 752x480
views of a textured plane (EuRoC.yaml calibration, 1200 features, scale 1.2, 8 levels,
FAST 20/7), a synthetic k=10 L=6 vocabulary of ORBvoc.txt's shape.  One step = extract L
and R, ComputeStereoMatches, ComputeBoW (levelsup 4), the close-point MapPoints, the RCCL
all-gather of every rank's keyframe slab, and SearchForTriangulation of each local
keyframe against its nn = 10 stream neighbours that pass LocalMapping's baseline test.

Prints ONE JSON line: value = keyframes/s over all ranks (max-over-ranks time); roofline of
the dominant extraction kernel; parity = every rank's keyframes (and the gathered copies of
their neighbours) and every one of their triangulation pair lists against the oracle;
cpu_baseline = the oracle (-O3 -march=native) doing one keyframe's work on the host's cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for _p in (ROOT, ROOT / "benchmarks"):
    if str(_p) not in sys.path:
        sys.path.insert(0, str(_p))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0


class OracleKeyFrames:
    """The oracle's version of every keyframe the parity check or the CPU baseline needs
    (extraction of L and R, ComputeStereoMatches, ComputeBoW, has-MapPoint), by window
    index, computed on demand on a thread pool."""

    def __init__(self, O, pl, vocab, window: int = 0):
        from orbslam2commentedbyxcm_amd.matcher import FrameView, feature_vector_csr
        self.O, self.pl, self.V = O, pl, vocab
        self.seq = pl.seqs[window]  # the keyframe window (texture) the checked step extracted
        s = pl.s
        self.p = O.params(s["nfeatures"], s["scale"], s["nlevels"], s["ini_th"], s["min_th"])
        self.FrameView, self.csr = FrameView, feature_vector_csr
        self.cache = {}

    def view(self, kl, dl, T, ur=None):
        s, sf = self.pl.s, self.pl.sf
        return self.FrameView(keys=kl, desc=dl, fx=s["fx"], fy=s["fy"], cx=s["cx"], cy=s["cy"], bf=s["bf"],
                              b=self.pl.mb, max_x=float(self.pl.W), max_y=float(self.pl.H), scale_factors=sf,
                              level_sigma2=sf * sf, Tcw=T, u_right=ur)

    def compute(self, g: int) -> dict:
        O, p, pl = self.O, self.p, self.pl
        left, right = self.seq.views([g])
        kl, dl, _ = O.extract(left[0], p)
        kr, dr, _ = O.extract(right[0], p)
        v = self.view(kl, dl, pl.poses[g])
        ur, dp = O.compute_stereo_matches(v, kr, dr, O.pyramid(left[0], p), O.pyramid(right[0], p), pl.s["fx"])
        bw, bv, fn, fo, fi = self.V.transform(dl, 4)
        has = ((ur >= 0) & (dp < np.float32(pl.th_depth))).astype(np.uint8)
        return {"kl": kl, "dl": dl, "kr": kr, "dr": dr, "ur": ur, "depth": dp, "fv": (fn, fo, fi), "has": has,
                "view": self.view(kl, dl, pl.poses[g], ur)}

    def fill(self, gs, threads: int):
        todo = [g for g in sorted(set(gs)) if g not in self.cache]
        with ThreadPoolExecutor(threads) as ex:
            for g, r in zip(todo, ex.map(self.compute, todo)):
                self.cache[g] = r

    def triangulate(self, g1: int, g2: int, F12):
        a, b = self.cache[g1], self.cache[g2]
        return self.O.search_for_triangulation(a["view"], a["has"], a["fv"], b["view"], b["has"], b["fv"], F12,
                                               False, False)


def _slab_fields(pl, buf: np.ndarray, rank: int, i: int) -> dict:
    """Host view of keyframe (rank, local i) in a gathered (or single) slab byte buffer."""
    from orbslam2commentedbyxcm_amd import KEYPOINT_DTYPE
    lay, cap = pl.lay, pl.cap

    def f(name, dt, count):
        o = rank * lay.nbytes + lay.offset[name] + i * lay.stride[name]
        return buf[o:o + count * np.dtype(dt).itemsize].view(dt)

    n = int(f("n", np.int32, 1)[0])
    nfv = int(f("nfv", np.int32, 1)[0])
    return {"n": n, "kl": f("kps", np.uint8, cap * 28).view(KEYPOINT_DTYPE)[:n], "dl": f("desc", np.uint8, cap * 32)
            .reshape(cap, 32)[:n], "ur": f("u_right", np.float32, cap)[:n], "has": f("has_mp", np.uint8, cap)[:n],
            "fn": f("fv_node", np.int32, cap)[:nfv], "fo": f("fv_off", np.int32, cap + 1)[:nfv + 1],
            "fi": f("fv_idx", np.int32, cap)}


def check(pl, ok: OracleKeyFrames, res: dict, nlocal: int, threads: int) -> dict:
    """This rank's first `nlocal` keyframes (every field the step writes), the gathered
    copies of their neighbours, and every pair list of theirs, bit-exact vs the oracle."""
    from orbslam2commentedbyxcm_amd.keyframes import record_index
    plan, B, world = pl.plan, pl.B, pl.world
    local_g = pl.local[:nlocal]
    sel = [p for p in range(len(plan.pairs)) if plan.kf1_window[p] in set(local_g)]
    need = set(local_g) | {int(plan.kf2_window[p]) for p in sel}
    ok.fill(need, threads)
    bad_kf, bad_pairs = [], []
    for i, g in enumerate(local_g):
        r = ok.cache[g]
        n = int(res["nl"][i])
        fn, fo, fi = r["fv"]
        good = (n == len(r["kl"]) and int(res["nr"][i]) == len(r["kr"])
                and np.array_equal(res["kl"][i, :n].view(np.uint8), r["kl"].view(np.uint8))
                and np.array_equal(res["dl"][i, :n], r["dl"])
                and np.array_equal(res["kr"][i, :len(r["kr"])].view(np.uint8), r["kr"].view(np.uint8))
                and np.array_equal(res["dr"][i, :len(r["kr"])], r["dr"])
                and np.array_equal(res["ur"][i, :n], r["ur"]) and np.array_equal(res["depth"][i, :n], r["depth"])
                and np.array_equal(res["has_mp"][i, :n], r["has"]) and int(res["nfv"][i]) == len(fn)
                and np.array_equal(res["fv_node"][i, :len(fn)], fn) and np.array_equal(res["fv_off"][i, :len(fo)], fo)
                and np.array_equal(res["fv_idx"][i, :fo[-1]], fi))
        if not good:
            bad_kf.append(g)
    bad_gathered = []
    if pl.collective:  # the neighbours as this rank received them over RCCL
        buf = res["gathered"]
        for h in sorted(need):
            q, i = h % world, h // world
            got, r = _slab_fields(pl, buf, q, i), ok.cache[h]
            fn, fo, fi = r["fv"]
            good = (got["n"] == len(r["kl"]) and np.array_equal(got["kl"].view(np.uint8), r["kl"].view(np.uint8))
                    and np.array_equal(got["dl"], r["dl"]) and np.array_equal(got["ur"], r["ur"])
                    and np.array_equal(got["has"], r["has"]) and np.array_equal(got["fn"], fn)
                    and np.array_equal(got["fo"], fo) and np.array_equal(got["fi"][:fo[-1]], fi))
            if not good:
                bad_gathered.append(h)
    with ThreadPoolExecutor(threads) as ex:
        refs = list(ex.map(lambda p: ok.triangulate(int(plan.kf1_window[p]), int(plan.kf2_window[p]), plan.F12[p]),
                           sel))
    npairs = []
    for p, ref in zip(sel, refs):
        n = int(res["tri_n"][p])
        npairs.append(len(ref))
        if n != len(ref) or not np.array_equal(res["tri_pairs"][p, :n], ref):
            bad_pairs.append(p)
        assert record_index(int(plan.kf1_window[p]), world, B) == plan.pairs[p, 0]
    return {"keyframes_checked": len(local_g), "keyframes_mismatched": len(bad_kf), "first_bad_keyframes": bad_kf[:8],
            "gathered_neighbours_checked": len(need) if pl.collective else 0,
            "gathered_mismatched": len(bad_gathered), "first_bad_gathered": bad_gathered[:8],
            "pairs_checked": len(sel), "pairs_mismatched": len(bad_pairs), "first_bad_pairs": bad_pairs[:8],
            "mean_triangulation_matches_ref": float(np.mean(npairs)) if npairs else 0.0,
            "bit_exact": not bad_kf and not bad_pairs and not bad_gathered}


def cpu_baseline(pl, O, text, seconds: float, threads: int) -> dict:
    """One keyframe's work on the host: extract L and R, ComputeStereoMatches, ComputeBoW
    and SearchForTriangulation against its planned neighbours (whose keyframe data is
    precomputed: it is their own keyframe's work), by the oracle built -O3 -march=native.
    Bounded sample: rank 0's first 32 keyframes, ~seconds/3 on one thread then ~seconds
    on `threads` threads."""
    flags = O.select("native")
    try:
        V = O.Vocab(text)
        ok = OracleKeyFrames(O, pl, V)
        sample = pl.local[:32]
        plan = pl.plan
        nb = {g: [(int(plan.kf2_window[p]), plan.F12[p]) for p in range(len(plan.pairs)) if plan.kf1_window[p] == g]
              for g in sample}
        ok.fill({h for g in sample for h, _ in nb[g]} | set(sample), threads)
        pre = dict(ok.cache)

        def one(g):
            r = ok.compute(g)  # the keyframe's own work, recomputed
            for h, F in nb[g]:
                b = pre[h]
                O.search_for_triangulation(r["view"], r["has"], r["fv"], b["view"], b["has"], b["fv"], F, False,
                                           False)

        def chain(start, stop, counter, idx):
            i = start
            while time.perf_counter() < stop:
                one(sample[i % len(sample)])
                counter[idx] += 1
                i += 1

        c1 = [0]
        t0 = time.perf_counter()
        chain(0, t0 + seconds / 3, c1, 0)
        el1 = time.perf_counter() - t0
        done = [0] * threads
        stop = time.perf_counter() + seconds
        t1 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(lambda t: chain(t, stop, done, t), range(threads)))
        el = time.perf_counter() - t1
    finally:
        O.select("parity")
    import bench
    npair = sum(len(v) for v in nb.values()) / len(nb)
    return {"value": round(sum(done) / el, 2), "unit": "keyframes/s", "cores": threads, "kind": "port",
            "single_thread_ms_per_keyframe": round(el1 * 1e3 / max(c1[0], 1), 3), "cpu_model": bench.cpu_model(),
            "flags": flags,
            "sample": f"{sum(done)} keyframes in {el:.1f}s on {threads} threads (+{c1[0]} in {el1:.1f}s on 1 thread), "
                      f"each = oracle C restatement of ORBextractor::operator() on L and R + ComputeStereoMatches + "
                      f"TemplatedVocabulary::transform + SearchForTriangulation against its {npair:.1f} planned "
                      f"neighbours (average), over 32 distinct keyframes; scalar port built {flags}"}


def parse(argv=None):
    ap = argparse.ArgumentParser(prog="bench.py --workload euroc")
    ap.add_argument("--workload", default="euroc")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="keyframes per rank per step")
    ap.add_argument("--nn", type=int, default=10, help="covisible neighbours (LocalMapping.cc:237, stereo)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--parity-frames", type=int, default=-1,
                    help="rank 0 keyframes to check (-1: all at world 1, 16 at world > 1; 0: none)")
    ap.add_argument("--level0-copy", action="store_true",
                    help="copy level 0 into the pyramids instead of reading it in place from the frames")
    ap.add_argument("--collective", action="store_true",
                    help="exchange the slabs through an RCCL process group even at --gpus 1 (a one-rank "
                         "all_gather_into_tensor into gathered buffers: the N-GPU data path on one GPU)")
    args, _ = ap.parse_known_args(argv)
    return args


def main(argv=None):
    args = parse(argv)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    collective = world > 1 or args.collective
    if collective:
        if world == 1:  # a one-rank group (env rendezvous: 127.0.0.1, a free port)
            import socket
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                with socket.socket() as sk:
                    sk.bind(("127.0.0.1", 0))
                    os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("nccl", device_id=dev)
    out = run(args, rank, world, local_rank, collective)
    if out is not None:
        print(json.dumps(out), flush=True)
    # every pipeline, extractor, matcher and vocabulary closed and the device synchronised
    # before the process group goes (r05e: an exit-time SIGSEGV, DESIGN.md §1 "Teardown")
    import bench
    bench.teardown(world if collective else 1, torch.device("cuda", local_rank))
    if collective and world == 1:
        dist.destroy_process_group()


def run(args, rank: int, world: int, device: int, collective: bool):
    """The configs[3] step on this rank, on GPU `device` (the process group, when
    collective, is already up): warmup, the timed steps (max over ranks), every rank's parity (counts summed)
    and bench line (None on the other ranks).  bench.py's headline run calls it at world
    size > 1 for its keyframe-exchange leg."""
    import torch
    import torch.distributed as dist

    from orbslam2commentedbyxcm_amd import ORBextractor, synth
    from orbslam2commentedbyxcm_amd.keyframes import EUROC, StereoKeyFramePipeline

    dev = torch.device("cuda", device)
    B = args.batch
    s = EUROC
    # the vocabulary's level-1 centres come from the stream's first left view (same on every rank)
    seq0 = synth.StereoSequence(3, 1, s["width"], s["height"], step=16, margin=256, disp=13)
    ex0 = ORBextractor(s["nfeatures"], s["scale"], s["nlevels"], s["ini_th"], s["min_th"], device=device)
    _, d0 = ex0(seq0.views([0])[0][0])
    del ex0
    t0 = time.perf_counter()
    text = synth.vocabulary_text(7, 10, 6, 0, 0, centres=d0)
    gen_s = time.perf_counter() - t0
    # A/B knobs of the bench (environment): keyframe sets, the right image's lane offset,
    # where the slab exchange is waited for
    pl = StereoKeyFramePipeline(B, rank, world, device=device, nn=args.nn, vocab_text=text,
                                nsets=int(os.environ.get("ORBX_KF_SETS", "4")),
                                lane_offset_stage=int(os.environ.get("ORBX_KF_LANE_OFFSET", "3")),
                                gather_async=os.environ.get("ORBX_GATHER_SYNC") != "1",
                                collective=collective, level0_in_place=not getattr(args, "level0_copy", False))

    def barrier():
        if world > 1:
            dist.barrier()

    pl.run(max(args.warmup, 2))
    torch.cuda.synchronize(dev)
    pl.set_timing(True)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    pl.run(args.steps)
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    value = B * world * args.steps / el
    stage_ms = pl.stage_times()
    pl.set_timing(False)
    res = pl.host_results()
    status_ok = pl.status()
    npairs_local = len(pl.plan.pairs)
    if world > 1:
        t = torch.tensor([npairs_local, pl.plan.skipped_baseline, int(res["tri_n"].sum())], dtype=torch.int64,
                         device=dev)
        dist.all_reduce(t)
        tot_pairs, tot_skipped, tot_matches = (int(x) for x in t.tolist())
    else:
        tot_pairs, tot_skipped, tot_matches = npairs_local, pl.plan.skipped_baseline, int(res["tri_n"].sum())

    out = None
    # every rank checks its own keyframes, the neighbours it received and its pair lists;
    # the counts are summed over the ranks
    parity = {"octree_status_clean": status_ok, "basis": __import__("bench").PARITY_BASIS}
    nchk = args.parity_frames if args.parity_frames >= 0 else (B if world == 1 else 16)
    threads = args.cpu_threads or __import__("bench").parity_threads(world)
    from oracle import oracle as O
    if nchk > 0:
        O.build()
        ok = OracleKeyFrames(O, pl, O.Vocab(text))
        parity.update(check(pl, ok, res, min(nchk, B), threads))
        keys = ("keyframes_checked", "keyframes_mismatched", "gathered_neighbours_checked", "gathered_mismatched",
                "pairs_checked", "pairs_mismatched")
        counts = [int(parity[k]) for k in keys] + [int(not status_ok), 1]
        if world > 1:
            t = torch.tensor(counts, dtype=torch.int64, device=dev)
            dist.all_reduce(t)
            counts = [int(x) for x in t.tolist()]
        parity.update({f"{k}_all_ranks": c for k, c in zip(keys, counts)})
        parity["ranks_checked"] = counts[-1]
        parity["bit_exact"] = counts[1] == 0 and counts[3] == 0 and counts[5] == 0 and counts[6] == 0
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(pl, O, text, args.cpu_seconds, threads)
        import bench
        n_mean = float(np.concatenate([res["nl"], res["nr"]]).mean())
        bytes_pf = bench.stage_bytes(pl.W, pl.H, n_mean)
        kern = {k: v for k, v in stage_ms.items() if k in bytes_pf and k != "total"}
        dom = bench.dominant_stage(kern, "euroc")
        achieved = bytes_pf[dom] * B / (stage_ms[dom] * 1e-3) / 1e9
        slab_mb = pl.lay.nbytes / 1e6
        out = {
            "metric": "keyframes/s stereo ORB extract (L+R) + ComputeStereoMatches + ComputeBoW + RCCL all-gather + "
                      "SearchForTriangulation vs covisible neighbours, 752x480 1200-feat (configs[3])",
            "value": round(value, 2),
            "unit": "keyframes/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "source_hash": __import__("bench").source_hash(),
            "config": {"workload": f"configs[3]: {B} stereo keyframes per GPU per step (keyframe g of the {B * world}-"
                                   f"keyframe window on rank g % {world}), synthetic rectified 752x480 views of a "
                                   f"textured plane at {pl.depth:.2f} m, EuRoC calibration, nFeatures=1200, scale 1.2, "
                                   f"8 levels, FAST 20/7, synthetic k=10 L=6 vocabulary; step = extract L+R, "
                                   f"ComputeStereoMatches, ComputeBoW(levelsup 4), close-point MapPoints, all-gather "
                                   f"of the keyframe slabs, SearchForTriangulation (ORBmatcher(0.6,false)) of each "
                                   f"keyframe vs its nn={args.nn} stream neighbours passing the baseline test",
                       "keyframes_per_gpu_step": B, "global_batch": B * world, "width": pl.W, "height": pl.H,
                       "parallelism": f"frame-sharded x{world} + all-gather", "slab_mb_per_rank": round(slab_mb, 2),
                       "extractor_sets": pl.nsets, "frame_row_pitch": int(pl.inputs[0][0].stride(1)),
                       "right_lane_offset_stage": int(os.environ.get("ORBX_KF_LANE_OFFSET", "3")),
                       "slab_exchange": ("none (world 1: slabs read in place)" if not collective else
                                         "rccl all_gather_into_tensor" if dist.get_backend() == "nccl" else
                                         "gloo all_gather, staged through host memory (one-GPU rehearsal)"),
                       "allgather_mb_per_rank_step": round(slab_mb * world, 2),
                       "triangulation_pairs_per_step": tot_pairs, "baseline_skipped_per_step": tot_skipped,
                       "triangulation_matches_per_step": tot_matches},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         **bench.profile_fields(dom, bytes_pf[dom] * B, stage_ms[dom], "euroc"),
                         "algorithmic_bytes_per_launch": int(bytes_pf[dom] * B),
                         "bytes_model": "SURVEY.md §8(d) per-stage algorithmic bytes per image x B images per launch",
                         "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
                         "concurrent_launches": 2, "frac_all_lanes": round(2 * achieved / HBM_PEAK_GBS, 5)},
            "cpu_baseline": cpu,
            "parity": parity,
            "mean_keypoints_per_image": round(n_mean, 1),
            "mean_stereo_matches_per_keyframe": round(float((res["ur"] >= 0).sum(axis=1).mean()), 1),
            "vocabulary_generate_s": round(gen_s, 2),
        }
    pl.close()
    return out


if __name__ == "__main__":
    main()
