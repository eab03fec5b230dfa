"""Exit-time teardown (DESIGN.md §1 "Teardown"; VERDICT r5 item 2: an exit-time SIGSEGV in
the C runtime's static destructors after a run that left HIP objects alive).

A process that exits with liborbx handle owners still alive -- held in a reference cycle,
so no refcount frees them -- must close every one of them from the atexit hook (before the
interpreter finalises, newest first, pipelines before the extractors and matchers they
hold), exactly once, and never from a __del__ running during finalisation.  The CPU test
drives the package's real Python classes over a stand-in for liborbx's C entry points
(recording every create / destroy); the GPU test runs real pipelines and exits without
closing them."""
import json
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]

FAKE = textwrap.dedent(r'''
    import ctypes as C, json, os, sys
    sys.path.insert(0, {root!r})
    from orbslam2commentedbyxcm_amd import _lib as L
    LOG = open({log!r}, "w")
    def rec(*ev):
        LOG.write(json.dumps([*ev, sys.is_finalizing()]) + "\n"); LOG.flush()
    class Fake:
        n = 0
        def _new(self, kind, out):
            Fake.n += 1
            out._obj.value = 0x1000 + Fake.n
            rec("create", kind, 0x1000 + Fake.n)
            return 0
        def orbx_extractor_create(self, prm, dev, out): return self._new("extractor", out)
        def orbx_matcher_create(self, dev, r, o, out): return self._new("matcher", out)
        def orbx_vocabulary_load_text(self, b, n, dev, out): return self._new("vocabulary", out)
        def orbx_stream_create(self, dev, k, prio, out): return self._new("stream", out)
        def orbx_extractor_destroy(self, h): rec("destroy", "extractor", h.value)
        def orbx_matcher_destroy(self, h): rec("destroy", "matcher", h.value)
        def orbx_vocabulary_destroy(self, h): rec("destroy", "vocabulary", h.value)
        def orbx_stream_destroy(self, h): rec("destroy", "stream", h.value); return 0
    L._lib = Fake()
    from orbslam2commentedbyxcm_amd import ORBextractor
    from orbslam2commentedbyxcm_amd.extractor import release_owned, stream_create
    from orbslam2commentedbyxcm_amd.matcher import ORBmatcher
    from orbslam2commentedbyxcm_amd.vocabulary import ORBVocabulary

    class SyncedStream:  # a torch stream object's synchronize()
        def __init__(self, h): self.h = h
        def synchronize(self): rec("sync", "stream", self.h)

    class Pipeline:  # the pipelines' shape: own stream, owners, release_owned in close()
        def __init__(self):
            self._own_ms = stream_create(0)
            self.ms = SyncedStream(self._own_ms)
            self.exs = [ORBextractor(1000, 1.2, 8, 20, 7), ORBextractor(1000, 1.2, 8, 20, 7)]
            self.matcher = ORBmatcher(0.9, True)
            L.track(self)
        def close(self):
            release_owned(self, [self.ms], [self.matcher, *self.exs], ["_own_ms"])
        def __del__(self, _fin=sys.is_finalizing):
            if not _fin():
                self.close()

    class Cycle:
        pass
    c = Cycle()
    c.me = c
    v = ORBVocabulary()
    assert v.loadFromText("k L")
    c.objs = [ORBextractor(500, 1.2, 8, 20, 7), v, Pipeline()]
    freed = ORBmatcher(0.6, True)  # freed normally: destroyed at once, not again at exit
    del freed
    rec("main_done", "-", 0)
    del c, v
''')


def _run(tmp_path):
    log = tmp_path / "log.jsonl"
    r = subprocess.run([sys.executable, "-c", FAKE.format(root=str(ROOT), log=str(log))], capture_output=True,
                       text=True, timeout=120)
    return r, [json.loads(x) for x in log.read_text().splitlines()]


def test_open_handles_closed_at_exit_in_order(tmp_path):
    r, ev = _run(tmp_path)
    assert r.returncode == 0, r.stderr
    created = [e[2] for e in ev if e[0] == "create"]
    destroyed = [e[2] for e in ev if e[0] == "destroy"]
    assert sorted(created) == sorted(destroyed) and len(set(destroyed)) == len(destroyed)  # all, once
    assert not any(e[3] for e in ev), "a handle was released during interpreter finalisation"
    done = [i for i, e in enumerate(ev) if e[0] == "main_done"][0]
    assert sum(e[0] == "destroy" for e in ev[:done]) == 1  # only the matcher freed by refcount
    tail = [e[:3] for e in ev[done + 1:]]
    kinds = {h: k for _, k, h in (e[:3] for e in ev if e[0] == "create")}
    # newest owner first: the pipeline (its stream synchronised, then its matcher and
    # extractors, then its stream destroyed), then the lone extractor, then the vocabulary
    # (registered when constructed, before that extractor)
    ms = [h for h, k in kinds.items() if k == "stream"][0]
    assert tail[0] == ["sync", "stream", ms]
    assert [kinds[h] for _, _, h in tail[1:4]] == ["matcher", "extractor", "extractor"]
    assert tail[4] == ["destroy", "stream", ms]
    assert [kinds[h] for _, _, h in tail[5:]] == ["extractor", "vocabulary"]


def test_close_is_idempotent_and_del_is_quiet(tmp_path):
    """Closing twice releases once; after close, __del__ releases nothing."""
    script = FAKE.replace("    del c, v\n", "    v.close(); v.close(); c.objs[2].close(); c.objs[2].close()\n"
                                              "    del c, v\n")
    log = tmp_path / "log2.jsonl"
    r = subprocess.run([sys.executable, "-c", script.format(root=str(ROOT), log=str(log))], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    ev = [json.loads(x) for x in log.read_text().splitlines()]
    destroyed = [e[2] for e in ev if e[0] == "destroy"]
    assert len(set(destroyed)) == len(destroyed) == sum(e[0] == "create" for e in ev)


@pytest.mark.gpu
def test_gpu_pipelines_left_open_exit_cleanly(orbx_built):
    """Real pipelines (monocular mid-step, stereo) and a vocabulary left open in a cycle: the
    process exits with status 0 and nothing on stderr about a fault."""
    script = textwrap.dedent(f'''
        import sys
        sys.path.insert(0, {str(ROOT)!r}); sys.path.insert(0, {str(ROOT / "benchmarks")!r})
        import faulthandler; faulthandler.enable()
        import numpy as np, torch
        from orbslam2commentedbyxcm_amd import synth
        from orbslam2commentedbyxcm_amd.pipeline import SequencePipeline, sequence_poses
        from orbslam2commentedbyxcm_amd.stereo import StereoSequencePipeline
        from orbslam2commentedbyxcm_amd.vocabulary import ORBVocabulary
        dev = torch.device("cuda", 0)
        f, off = synth.sequence(1, 8)
        d_f, d_T = torch.from_numpy(f).to(dev), torch.from_numpy(sequence_poses(off)).to(dev)
        a = SequencePipeline(8, 640, 480)
        a.step(d_f, d_T)          # left mid-pipeline: one batch extracted, not matched
        s = StereoSequencePipeline(4, 640, 480, 500.0, 500.0, 320.0, 240.0, 40.0, params=(1000, 1.2, 8, 20, 7),
                                   track=False)
        s.step(d_f[:4], d_f[4:])
        v = ORBVocabulary(); assert v.loadFromText(synth.vocabulary_text(1, 5, 3))
        class C: pass
        c = C(); c.me = c; c.objs = [a, s, v]
        print("stepped", flush=True)
    ''')
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "stepped" in r.stdout, (r.returncode, r.stderr[-2000:])
    assert "Fatal Python error" not in r.stderr and "SIGSEGV" not in r.stderr, r.stderr[-2000:]
