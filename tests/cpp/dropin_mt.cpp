// Concurrent drop-in calls from C++ (what an unchanged, multi-instance Tracking.cc pays,
// without Python in the way): T threads, each with its own ORBextractor and two
// ORBmatchers (include/orbx.hpp; each instance owns its stream and pinned staging), run
// per frame ORBextractor::operator() on a C1 image (ORBextractor.cc:1513-1629),
// SearchByProjection(Frame&, const Frame&, th, bMono) (a12, ORBmatcher.cc:1620-1789) and
// SearchByProjection(Frame&, vector<MapPoint*>, th) (a11, cc:61-173) on host arrays, for
// a fixed wall time.  Frame k of a thread extracts image (k + thread) % M of the scene's M
// images, and EVERY frame's keypoints, descriptors and both searches' outputs are compared
// with the oracle's (precomputed per image in the scene file).
//   dropin_mt <scene.bin> <threads> <seconds>
// prints one JSON object: {"threads": T, "frames": N, "seconds": s, "frames_per_s": r,
//   "frames_checked": C, "frames_mismatched": X, "bit_exact": b}
// scene.bin is written by benchmarks/dropin_bench.py (layout in write_scene there).
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "orbx.hpp"

namespace {

struct Reader {
    FILE* f;
    template <typename T>
    std::vector<T> vec(size_t n) {
        std::vector<T> v(n);
        if (n && std::fread(v.data(), sizeof(T), n, f) != n) throw std::runtime_error("short scene file");
        return v;
    }
    template <typename T>
    T one() {
        return vec<T>(1)[0];
    }
};

struct Scene {
    int W, H, nA, nB, L, nq;
    float fx, fy, cx, cy;
    std::vector<orbx_keypoint> kA, kB;
    std::vector<uint8_t> dA, dB;
    std::vector<float> TA, TB, sf, sg;
    std::vector<float> pos;
    std::vector<uint8_t> mdesc, bad;
    std::vector<int32_t> obs;
    std::vector<uint8_t> in_view;
    std::vector<float> px, py, pxr, vcos;
    std::vector<int32_t> slev, queries, last_mp;
    int32_t n12, n11;
    std::vector<int32_t> c_ref, f_ref;
    std::vector<std::vector<uint8_t>> img;     // the M images
    std::vector<std::vector<orbx_keypoint>> k_ref;  // the oracle's keypoints / descriptors per image
    std::vector<std::vector<uint8_t>> d_ref;
};

Scene load(const char* path) {
    Scene s;
    Reader r{std::fopen(path, "rb")};
    if (!r.f) throw std::runtime_error("cannot open scene file");
    s.W = r.one<int32_t>(), s.H = r.one<int32_t>(), s.nA = r.one<int32_t>(), s.nB = r.one<int32_t>();
    s.L = r.one<int32_t>(), s.nq = r.one<int32_t>();
    s.fx = r.one<float>(), s.fy = r.one<float>(), s.cx = r.one<float>(), s.cy = r.one<float>();
    s.kA = r.vec<orbx_keypoint>(s.nA), s.dA = r.vec<uint8_t>((size_t)s.nA * 32), s.TA = r.vec<float>(12);
    s.kB = r.vec<orbx_keypoint>(s.nB), s.dB = r.vec<uint8_t>((size_t)s.nB * 32), s.TB = r.vec<float>(12);
    s.sf = r.vec<float>(s.L), s.sg = r.vec<float>(s.L);
    s.pos = r.vec<float>((size_t)s.nA * 3), s.mdesc = r.vec<uint8_t>((size_t)s.nA * 32);
    s.obs = r.vec<int32_t>(s.nA), s.bad = r.vec<uint8_t>(s.nA);
    s.in_view = r.vec<uint8_t>(s.nA), s.px = r.vec<float>(s.nA), s.py = r.vec<float>(s.nA);
    s.pxr = r.vec<float>(s.nA), s.slev = r.vec<int32_t>(s.nA), s.vcos = r.vec<float>(s.nA);
    s.queries = r.vec<int32_t>(s.nq), s.last_mp = r.vec<int32_t>(s.nA);
    s.n12 = r.one<int32_t>(), s.c_ref = r.vec<int32_t>(s.nB);
    s.n11 = r.one<int32_t>(), s.f_ref = r.vec<int32_t>(s.nB);
    const int M = r.one<int32_t>();
    if (M < 1) throw std::runtime_error("no images in the scene file");
    for (int j = 0; j < M; j++) {
        s.img.push_back(r.vec<uint8_t>((size_t)s.W * s.H));
        const int nk = r.one<int32_t>();
        s.k_ref.push_back(r.vec<orbx_keypoint>(nk));
        s.d_ref.push_back(r.vec<uint8_t>((size_t)nk * 32));
    }
    std::fclose(r.f);
    return s;
}

orbx_frame_view view(const Scene& s, bool a) {
    orbx_frame_view v{};
    v.n = a ? s.nA : s.nB;
    v.keys = a ? s.kA.data() : s.kB.data();
    v.desc = a ? s.dA.data() : s.dB.data();
    v.u_right = nullptr;
    v.fx = s.fx, v.fy = s.fy, v.cx = s.cx, v.cy = s.cy, v.bf = 0.f, v.b = 0.f;
    v.min_x = 0.f, v.max_x = (float)s.W, v.min_y = 0.f, v.max_y = (float)s.H;
    v.nlevels = s.L;
    v.scale_factors = s.sf.data();
    v.level_sigma2 = s.sg.data();
    std::memcpy(v.Tcw, a ? s.TA.data() : s.TB.data(), sizeof(v.Tcw));
    return v;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 4) {
        std::fprintf(stderr, "usage: %s scene.bin threads seconds\n", argv[0]);
        return 2;
    }
    const int T = std::atoi(argv[2]);
    const double seconds = std::atof(argv[3]);
    try {
        const Scene s = load(argv[1]);
        const orbx_frame_view A = view(s, true), B = view(s, false);
        orbx_mappoints mps{};
        mps.n = s.nA, mps.pos = s.pos.data(), mps.desc = s.mdesc.data(), mps.observations = s.obs.data();
        mps.bad = s.bad.data();
        orbx_track trk{};
        trk.in_view = s.in_view.data(), trk.proj_x = s.px.data(), trk.proj_y = s.py.data();
        trk.proj_xr = s.pxr.data(), trk.scale_level = s.slev.data(), trk.view_cos = s.vcos.data();

        std::atomic<int> ready{0};
        std::atomic<bool> go{false};
        std::atomic<long> frames{0}, checked{0}, mismatched{0};
        std::atomic<int> failed{0};
        std::chrono::steady_clock::time_point t_end;
        std::vector<double> span_start(T), span_end(T);
        const auto t_ref = std::chrono::steady_clock::now();
        auto worker = [&](int i) {
            try {
                orbx::ORBextractor ex(1000, 1.2f, 8, 20, 7);
                orbx::ORBmatcher m12(0.9f, true), m11(0.8f, false);
                std::vector<orbx_keypoint> kps;
                std::vector<uint8_t> desc;
                std::vector<int32_t> cur(s.nB), loc(s.nB);
                const int M = (int)s.img.size();
                long k = i;  // this thread's frame counter (threads start on different images)
                auto frame = [&]() -> bool {
                    const int j = (int)(k++ % M);
                    ex(s.img[j].data(), s.W, s.H, (size_t)s.W, kps, desc);
                    std::fill(cur.begin(), cur.end(), -1);
                    const int n12 = m12.SearchByProjection(B, cur.data(), A, s.last_mp.data(), nullptr, mps, 15.f, true);
                    std::fill(loc.begin(), loc.end(), -1);
                    const int n11 = m11.SearchByProjection(B, loc.data(), s.queries, mps, trk, 3.f);
                    return kps.size() == s.k_ref[j].size() &&
                           std::memcmp(kps.data(), s.k_ref[j].data(), kps.size() * sizeof(orbx_keypoint)) == 0 &&
                           desc == s.d_ref[j] && n12 == s.n12 && cur == s.c_ref && n11 == s.n11 && loc == s.f_ref;
                };
                long bad = 0, n_chk = 0;
                for (int w = 0; w < 2; w++, n_chk++) bad += !frame();  // warm-up (checked too)
                ready++;
                while (!go.load()) std::this_thread::yield();
                const auto t0 = std::chrono::steady_clock::now();
                long n = 0;
                while (std::chrono::steady_clock::now() < t_end) {
                    bad += !frame();  // every frame compared
                    n++;
                }
                n_chk += n;
                checked += n_chk;
                mismatched += bad;
                const auto t1 = std::chrono::steady_clock::now();
                span_start[i] = std::chrono::duration<double>(t0 - t_ref).count();
                span_end[i] = std::chrono::duration<double>(t1 - t_ref).count();
                frames += n;
            } catch (const std::exception& e) {
                std::fprintf(stderr, "thread %d: %s\n", i, e.what());
                failed++;
                ready++;
            }
        };
        std::vector<std::thread> th;
        for (int i = 0; i < T; i++) th.emplace_back(worker, i);
        while (ready.load() < T) std::this_thread::sleep_for(std::chrono::milliseconds(1));
        t_end = std::chrono::steady_clock::now() + std::chrono::microseconds((long)(seconds * 1e6));
        go = true;
        for (auto& t : th) t.join();
        if (failed.load()) return 1;
        double a = 1e30, b = 0;
        for (int i = 0; i < T; i++) {
            a = span_start[i] < a ? span_start[i] : a;
            b = span_end[i] > b ? span_end[i] : b;
        }
        const double el = b - a;
        std::printf("{\"threads\": %d, \"frames\": %ld, \"seconds\": %.4f, \"frames_per_s\": %.1f, "
                    "\"frames_checked\": %ld, \"frames_mismatched\": %ld, \"images\": %d, \"bit_exact\": %s}\n",
                    T, frames.load(), el, frames.load() / el, checked.load(), mismatched.load(), (int)s.img.size(),
                    mismatched.load() ? "false" : "true");
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
