// TEST INFRASTRUCTURE (H1 measurement): DistributeOctTree's node list
// and final-phase sort run under glibc malloc, so that equal-size nodes are ordered by the
// heap addresses glibc itself hands out, as in the reference's process.
//
// This is a transcription of the allocation behaviour of ORBextractor::DistributeOctTree
// (ORBextractor.cc:667-1013) and ExtractorNode::DivideNode (cc:581-653): a std::list of
// nodes whose member layout matches ExtractorNode (ORBextractor.h:41-62: a vector of
// 28-byte keypoints, four int points, a list iterator and a bool -- 72 bytes, so a list
// node is an 88-byte malloc request like the reference's), children built as locals
// with reserve(parent size), copied into the list by push_front, the parent erased, and
// the final phase sorting (size, node pointer) pairs with std::sort and splitting from
// the back (cc:899-913).  The keypoint geometry, which decides nothing but the tie order
// here, follows the C oracle (oracle/orbx_oracle.c ora_distribute_octree), which the GPU
// kernel is checked against.
//
// Input (stdin-named file): int32 nframes, nlevels, nfeatures, mode, thread; then per frame
// and level: int32 minX, maxX, minY, maxY, N, ncells, ncand, ncells x (int32 count,
// int32 second_try), ncand x (float x, float y, float response).
// Output: per frame and level: int32 nkept, then nkept x (float x, float y, float response).
// mode 0: the octree's own allocations only; mode 1: also the surrounding per-frame
// allocations of ORBextractor::operator() (pyramid and descriptor Mats: OpenCV's
// StdMatAllocator data block + an 88-byte UMatData each; the level's vToDistributeKeys,
// the per-cell FAST vectors, allKeypoints, the output keypoints).
// thread 1: run in a std::thread (a non-main malloc arena, as ORB-SLAM2's Tracking thread).
// mode 2: the octree's own allocations from a monotonic bump allocator (global operator
// new replaced; delete frees nothing), reset at every level: a node created later always
// has a higher address, which is the order SURVEY.md App. A H1 names and the oracle ships
// ("later-created node splits first"), so this mode must equal the oracle on every level,
// tie-deciding or not -- the check of the transcription on the levels glibc leaves open.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <list>
#include <new>
#include <thread>
#include <utility>
#include <vector>

namespace {
constexpr size_t kArenaBytes = size_t(512) << 20;
char* g_arena = nullptr;
size_t g_top = 0;
bool g_bump = false;  // operator new bumps from g_arena (mode 2, while a level is distributed)

void* bump(size_t n) {
    const size_t at = (g_top + 15) & ~size_t(15);
    if (at + n > kArenaBytes) {
        std::fprintf(stderr, "bump arena exhausted\n");
        std::abort();
    }
    g_top = at + n;
    return g_arena + at;
}
bool in_arena(void* p) { return g_arena && (char*)p >= g_arena && (char*)p < g_arena + kArenaBytes; }
}  // namespace

// Outside mode 2 these forward to malloc / free, as the default operator new does, so the
// glibc modes see the same requests as before.
void* operator new(size_t n) {
    if (g_bump) return bump(n ? n : 1);
    void* p = std::malloc(n ? n : 1);
    if (!p) throw std::bad_alloc();
    return p;
}
void operator delete(void* p) noexcept {
    if (p && !in_arena(p)) std::free(p);
}
void operator delete(void* p, size_t) noexcept {
    if (p && !in_arena(p)) std::free(p);
}

struct KP28 {  // cv::KeyPoint: pt, size, angle, response, octave, class_id (28 bytes)
    float x, y, size, angle, response;
    int octave, class_id;
};
static_assert(sizeof(KP28) == 28, "cv::KeyPoint is 28 bytes");

struct Pt {
    int x, y;
};

struct Quad;
using QuadList = std::list<Quad>;

struct Quad {  // member order and sizes of ExtractorNode
    std::vector<KP28> keys;
    Pt ul, ur, bl, br;
    QuadList::iterator self;
    bool leaf = false;

    void split(Quad& a, Quad& b, Quad& c, Quad& d) const {
        const int hx = (int)std::ceil((float)(ur.x - ul.x) / 2);
        const int hy = (int)std::ceil((float)(br.y - ul.y) / 2);
        a.ul = ul; a.ur = {ul.x + hx, ul.y}; a.bl = {ul.x, ul.y + hy}; a.br = {ul.x + hx, ul.y + hy};
        b.ul = a.ur; b.ur = ur; b.bl = a.br; b.br = {ur.x, ul.y + hy};
        c.ul = a.bl; c.ur = a.br; c.bl = bl; c.br = {a.br.x, bl.y};
        d.ul = c.ur; d.ur = b.br; d.bl = c.br; d.br = br;
        a.keys.reserve(keys.size());
        b.keys.reserve(keys.size());
        c.keys.reserve(keys.size());
        d.keys.reserve(keys.size());
        for (const KP28& k : keys) {
            if (k.x < a.ur.x) (k.y < a.br.y ? a : c).keys.push_back(k);
            else (k.y < a.br.y ? b : d).keys.push_back(k);
        }
        for (Quad* q : {&a, &b, &c, &d})
            if (q->keys.size() == 1) q->leaf = true;
    }
};

using SizePtr = std::pair<int, Quad*>;

// push the non-empty children to the front (a, b, c, d in turn), recording the splittable ones
static void push_children(QuadList& lst, Quad& a, Quad& b, Quad& c, Quad& d, std::vector<SizePtr>& grow,
                          int* expand) {
    for (Quad* q : {&a, &b, &c, &d}) {
        if (q->keys.empty()) continue;
        lst.push_front(*q);
        if (q->keys.size() > 1) {
            if (expand) (*expand)++;
            grow.push_back(std::make_pair((int)q->keys.size(), &lst.front()));
            lst.front().self = lst.begin();
        }
    }
}

static std::vector<KP28> distribute(const std::vector<KP28>& in, int minX, int maxX, int minY, int maxY, int N,
                                    int nfeatures) {
    const int nIni = (int)std::round((float)(maxX - minX) / (maxY - minY));
    const float hX = (float)(maxX - minX) / nIni;
    QuadList lst;
    std::vector<Quad*> ini;
    ini.resize(nIni);
    for (int i = 0; i < nIni; i++) {
        Quad q;
        q.ul = {(int)(hX * (float)i), 0};
        q.ur = {(int)(hX * (float)(i + 1)), 0};
        q.bl = {q.ul.x, maxY - minY};
        q.br = {q.ur.x, maxY - minY};
        q.keys.reserve(in.size());
        lst.push_back(q);
        ini[i] = &lst.back();
    }
    for (const KP28& k : in) ini[(int)(k.x / hX)]->keys.push_back(k);
    for (auto it = lst.begin(); it != lst.end();) {
        if (it->keys.size() == 1) {
            it->leaf = true;
            ++it;
        } else if (it->keys.empty()) {
            it = lst.erase(it);
        } else {
            ++it;
        }
    }
    bool done = false;
    std::vector<SizePtr> grow;
    grow.reserve(lst.size() * 4);
    while (!done) {
        int prev = (int)lst.size();
        int expand = 0;
        grow.clear();
        for (auto it = lst.begin(); it != lst.end();) {
            if (it->leaf) {
                ++it;
                continue;
            }
            Quad a, b, c, d;
            it->split(a, b, c, d);
            push_children(lst, a, b, c, d, grow, &expand);
            it = lst.erase(it);
        }
        if ((int)lst.size() >= N || (int)lst.size() == prev) {
            done = true;
        } else if ((int)lst.size() + expand * 3 > N) {
            while (!done) {
                prev = (int)lst.size();
                std::vector<SizePtr> last = grow;
                grow.clear();
                std::sort(last.begin(), last.end());  // ties: by node address (H1)
                for (int j = (int)last.size() - 1; j >= 0; j--) {
                    Quad a, b, c, d;
                    last[j].second->split(a, b, c, d);
                    push_children(lst, a, b, c, d, grow, nullptr);
                    lst.erase(last[j].second->self);
                    if ((int)lst.size() >= N) break;
                }
                if ((int)lst.size() >= N || (int)lst.size() == prev) done = true;
            }
        }
    }
    std::vector<KP28> out;
    out.reserve(nfeatures);
    for (Quad& q : lst) {
        const KP28* best = &q.keys[0];
        for (size_t k = 1; k < q.keys.size(); k++)
            if (q.keys[k].response > best->response) best = &q.keys[k];
        out.push_back(*best);
    }
    return out;
}

// cv::Mat data under OpenCV 3.x's StdMatAllocator: fastMalloc(total) (16-byte aligned,
// one pointer of bookkeeping) and then `new UMatData` (88 bytes); released data first.
struct MatBuf {
    void* data = nullptr;
    void* u = nullptr;
    void make(size_t bytes) {
        release();
        data = std::malloc(bytes + sizeof(void*) + 16);
        u = std::malloc(88);
    }
    void release() {
        if (data) {
            std::free(data);
            std::free(u);
        }
        data = u = nullptr;
    }
};

struct LevelIn {
    int minX, maxX, minY, maxY, N;
    std::vector<int> cell_count, cell_second;
    std::vector<KP28> cand;
    int w, h;
};

static int rd(FILE* f) {
    int v;
    if (std::fread(&v, 4, 1, f) != 1) std::exit(3);
    return v;
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    FILE* fi = std::fopen(argv[1], "rb");
    FILE* fo = std::fopen(argv[2], "wb");
    if (!fi || !fo) return 2;
    const int nframes = rd(fi), nlevels = rd(fi), nfeatures = rd(fi), mode = rd(fi), thread = rd(fi);
    std::vector<std::vector<LevelIn>> frames(nframes, std::vector<LevelIn>(nlevels));
    for (auto& fr : frames)
        for (auto& L : fr) {
            L.minX = rd(fi); L.maxX = rd(fi); L.minY = rd(fi); L.maxY = rd(fi); L.N = rd(fi);
            const int nc = rd(fi), nk = rd(fi);
            L.w = rd(fi); L.h = rd(fi);
            L.cell_count.resize(nc);
            L.cell_second.resize(nc);
            for (int c = 0; c < nc; c++) {
                L.cell_count[c] = rd(fi);
                L.cell_second[c] = rd(fi);
            }
            L.cand.resize(nk);
            for (int k = 0; k < nk; k++) {
                float v[3];
                if (std::fread(v, 4, 3, fi) != 3) return 3;
                L.cand[k] = KP28{v[0], v[1], 7.f, -1.f, v[2], 0, -1};
            }
        }
    std::fclose(fi);
    if (mode == 2) {
        g_arena = (char*)std::malloc(kArenaBytes);
        if (!g_arena) return 4;
    }
    std::vector<std::vector<std::vector<KP28>>> result(nframes);
    auto run = [&]() {
        std::vector<MatBuf> pyr(nlevels);
        MatBuf desc_prev, desc_cur;
        std::vector<KP28> kps_prev;
        for (int f = 0; f < nframes; f++) {
            if (mode == 1)  // ComputePyramid: a new bordered Mat per level replaces last frame's
                for (int l = 0; l < nlevels; l++) {
                    MatBuf nb;
                    nb.make((size_t)(frames[f][l].w + 38) * (frames[f][l].h + 38));
                    pyr[l].release();
                    pyr[l] = nb;
                }
            std::vector<std::vector<KP28>> all;
            all.resize(nlevels);
            for (int l = 0; l < nlevels; l++) {
                const LevelIn& L = frames[f][l];
                std::vector<KP28> todist;
                if (mode == 1) {
                    todist.reserve((size_t)nfeatures * 10);
                    size_t k = 0;
                    for (size_t c = 0; c < L.cell_count.size(); c++) {
                        std::vector<KP28> cell;  // cv::FAST's output vector (push_back growth)
                        const int n = L.cell_count[c];
                        if (L.cell_second[c]) cell.clear();  // first threshold found nothing
                        for (int i = 0; i < n; i++) cell.push_back(L.cand[k + i]);
                        for (const KP28& p : cell) todist.push_back(p);
                        k += n;
                    }
                } else {
                    todist = L.cand;
                }
                if (mode == 2) {  // bump-allocated octree, written out before the arena is reused
                    g_top = 0;
                    g_bump = true;
                    std::vector<KP28> keep = distribute(todist, L.minX, L.maxX, L.minY, L.maxY, L.N, nfeatures);
                    g_bump = false;
                    const int n = (int)keep.size();
                    std::fwrite(&n, 4, 1, fo);
                    for (const KP28& k : keep) {
                        const float v[3] = {k.x, k.y, k.response};
                        std::fwrite(v, 4, 3, fo);
                    }
                    continue;
                }
                std::vector<KP28>& keep = all[l];
                keep.reserve(nfeatures);
                keep = distribute(todist, L.minX, L.maxX, L.minY, L.maxY, L.N, nfeatures);
                result[f].push_back(keep);
            }
            if (mode == 1) {  // operator(): descriptors, output keypoints, a blurred clone per level
                size_t n = 0;
                for (auto& v : all) n += v.size();
                desc_cur.make(n * 32);
                std::vector<KP28> out;
                out.reserve(n);
                for (int l = 0; l < nlevels; l++) {
                    MatBuf work;
                    work.make((size_t)frames[f][l].w * frames[f][l].h);
                    out.insert(out.end(), all[l].begin(), all[l].end());
                    work.release();
                }
                desc_prev.release();  // the previous Frame's outputs die with it
                std::swap(desc_prev, desc_cur);
                kps_prev.swap(out);
            }
        }
        for (auto& p : pyr) p.release();
        desc_prev.release();
    };
    if (thread) {
        std::thread t(run);
        t.join();
    } else {
        run();
    }
    for (auto& fr : result)
        for (auto& lv : fr) {
            const int n = (int)lv.size();
            std::fwrite(&n, 4, 1, fo);
            for (const KP28& k : lv) {
                const float v[3] = {k.x, k.y, k.response};
                std::fwrite(v, 4, 3, fo);
            }
        }
    std::fclose(fo);
    return 0;
}
