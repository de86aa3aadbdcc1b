// planar_prior.cpp -- host side of the planar-prior pass.
//
// Restates ACMMP::GetSupportPoints / DelaunayTriangulation / GetPriorPlaneParams /
// GetDepthFromPlaneParam (ACMMP.cpp:904-1011) and the triangle rasterisation + prior-depth
// mask of ProcessProblem (main.cpp:113-181) without OpenCV.  Runs on the host (the reference
// runs it on the host too); compiled with -ffp-contract=off, float/double exactly where the
// reference's C++ promotes.
//
// Delaunay: divide and conquer (Guibas-Stolfi merges, Dwyer's strips; parallel over host threads) on
// the integer support points with exact predicates (64-bit orientation, 64/128-bit in-circle); an
// incremental Bowyer-Watson form is its fallback.  cv::Subdiv2D's triangle order and its choice among
// co-circular configurations are not reproduced -- that part is "parity unpinned" (SURVEY.md §8c):
// the device side is pinned by injecting prior planes + masks (acmmp_set_planar_prior).
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <thread>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <cstdlib>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <vector>

#include "acmmp.h"
#include "planar.h"

namespace {

constexpr double kMPi = 3.14159265358979323846;  // M_PI

struct Pt { long long x, y; };

inline int incircle128(const Pt& a, const Pt& b, const Pt& c, const Pt& d) {
    typedef __int128 i128;
    const i128 adx = a.x - d.x, ady = a.y - d.y, bdx = b.x - d.x, bdy = b.y - d.y, cdx = c.x - d.x, cdy = c.y - d.y;
    const i128 ad = adx * adx + ady * ady, bd = bdx * bdx + bdy * bdy, cd = cdx * cdx + cdy * cdy;
    const i128 det = ad * (bdx * cdy - bdy * cdx) - bd * (adx * cdy - ady * cdx) + cd * (adx * bdy - ady * bdx);
    return det > 0 ? 1 : (det < 0 ? -1 : 0);
}

inline long long orient(const Pt& a, const Pt& b, const Pt& c) {
    return (b.x - a.x) * (c.y - a.y) - (b.y - a.y) * (c.x - a.x);
}

// > 0 when d lies strictly inside the circumcircle of the counter-clockwise triangle (a, b, c).
// Exact either way: 64-bit when every coordinate difference is below 2^14 in magnitude (terms below
// 2^59, so the three-term sum stays below 2^63), 128-bit otherwise (the super triangle's vertices).
inline int incircle(const Pt& a, const Pt& b, const Pt& c, const Pt& d) {
    const long long adx = a.x - d.x, ady = a.y - d.y, bdx = b.x - d.x, bdy = b.y - d.y, cdx = c.x - d.x,
                    cdy = c.y - d.y;
    const long long lim = 1ll << 14;
    if (std::llabs(adx) < lim && std::llabs(ady) < lim && std::llabs(bdx) < lim && std::llabs(bdy) < lim &&
        std::llabs(cdx) < lim && std::llabs(cdy) < lim) {
        const long long ad = adx * adx + ady * ady, bd = bdx * bdx + bdy * bdy, cd = cdx * cdx + cdy * cdy;
        const long long det = ad * (bdx * cdy - bdy * cdx) - bd * (adx * cdy - ady * cdx) + cd * (adx * bdy - ady * bdx);
        return det > 0 ? 1 : (det < 0 ? -1 : 0);
    }
    return incircle128(a, b, c, d);
}

struct Tri {
    int v[3];     // counter-clockwise
    int nb[3];    // neighbour across the edge opposite v[i]; -1 = none
    bool alive;
};

// Host worker threads shared by every planar-prior call of the process: run(n, f) calls f(0 .. n-1) on the
// pool's workers and the calling thread and returns when all have returned.  A call spawned ~100 std::threads
// (the Delaunay strips, the merges' halves, the triangle scan, the plane fits) -- milliseconds of thread creation
// per call, with three pipeline contexts calling at once.  The caller takes its own job's tasks too, so a task
// may call run() itself (the merges nest) without waiting on a busy pool.
class HostPool {
public:
    static HostPool& get() {
        static HostPool* p = new HostPool();               // never destroyed: the workers outlive static destructors
        return *p;
    }
    template <typename F>
    void run(int n, F&& f) {
        if (n <= 1 || workers_ == 0) {
            for (int t = 0; t < n; ++t) f(t);
            return;
        }
        Job job;
        job.n = n;
        job.fn = [&f](int t) { f(t); };
        {
            std::lock_guard<std::mutex> g(mu_);
            jobs_.push_back(&job);
        }
        cv_.notify_all();
        for (int t; (t = job.next.fetch_add(1)) < n;) {
            job.fn(t);
            job.done.fetch_add(1);
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            jobs_.erase(std::find(jobs_.begin(), jobs_.end(), &job));
        }
        while (job.done.load() < n) std::this_thread::yield();   // workers finishing this job's last tasks
    }
    int threads() const { return workers_ + 1; }

private:
    struct Job {
        int n = 0;
        std::function<void(int)> fn;
        std::atomic<int> next{0}, done{0};
    };
    HostPool() {
        const unsigned hw = std::thread::hardware_concurrency();
        workers_ = static_cast<int>(std::min<unsigned>(hw ? hw : 1, 16u)) - 1;
        for (int k = 0; k < workers_; ++k) std::thread([this] { work(); }).detach();
    }
    void work() {
        for (;;) {
            Job* j = nullptr;
            int t = 0;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] {
                    for (Job* x : jobs_)
                        if (x->next.load() < x->n) return true;
                    return false;
                });
                for (Job* x : jobs_) {
                    t = x->next.fetch_add(1);
                    if (t < x->n) { j = x; break; }
                }
            }
            if (j) {
                j->fn(t);
                j->done.fetch_add(1);
            }
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<Job*> jobs_;
    int workers_ = 0;
};

class Delaunay {
public:
    explicit Delaunay(std::vector<Pt> pts, long long extent) : p_(std::move(pts)) {
        const long long M = extent * 4096 + 1024;        // super triangle, far outside the image
        n_real_ = static_cast<int>(p_.size());
        p_.push_back({-M, -M});
        p_.push_back({3 * M, -M});
        p_.push_back({-M, 3 * M});
        t_.reserve(2 * static_cast<size_t>(n_real_) + 16);        // a triangulation of n points: < 2n + 1 triangles
        mark_.reserve(t_.capacity());
        t_.push_back({{n_real_, n_real_ + 1, n_real_ + 2}, {-1, -1, -1}, true});
    }

    // Points go in along a Hilbert curve over the image: each insertion's walk and cavity stay local.
    // (In the support points' own order -- 5-pixel column strips -- every point at the head of a strip
    // re-triangulated the whole previous strip's hull fan: 36k points took 0.45 s, 112k 6 s.)  The
    // Delaunay triangulation does not depend on the order except among co-circular points, whose
    // diagonal any order may pick (cv::Subdiv2D's choice is not reproduced either).
    void run() {
        std::vector<std::pair<uint64_t, int>> key(n_real_);
        long long ext = 1;
        for (int i = 0; i < n_real_; ++i) ext = std::max(ext, std::max(p_[i].x, p_[i].y) + 1);
        int bits = 1;
        while ((1ll << bits) < ext) ++bits;
        for (int i = 0; i < n_real_; ++i) key[i] = {hilbert(bits, p_[i].x, p_[i].y), i};
        std::sort(key.begin(), key.end());
        for (const auto& k : key) insert(k.second);
    }

    // triangles without super vertices, each rotated to start at its lowest point index (orientation
    // kept) and listed in increasing (v0, v1, v2): an order that depends on the triangle set only
    // (a counting sort on v0, then the few triangles sharing a v0 by (v1, v2): std::sort of the whole list
    // took 12-17 ms of a 2000x1500 view's 65)
    std::vector<std::array<int, 3>> triangles() const {
        std::vector<int> start(static_cast<size_t>(n_real_) + 1, 0);
        for (const Tri& t : t_) {
            if (!t.alive || t.v[0] >= n_real_ || t.v[1] >= n_real_ || t.v[2] >= n_real_) continue;
            ++start[std::min(t.v[0], std::min(t.v[1], t.v[2])) + 1];
        }
        for (int i = 0; i < n_real_; ++i) start[i + 1] += start[i];
        std::vector<std::array<int, 3>> out(static_cast<size_t>(start[n_real_]));
        std::vector<int> fill(start.begin(), start.end() - 1);
        for (const Tri& t : t_) {
            if (!t.alive || t.v[0] >= n_real_ || t.v[1] >= n_real_ || t.v[2] >= n_real_) continue;
            int r = 0;
            if (t.v[1] < t.v[r]) r = 1;
            if (t.v[2] < t.v[r]) r = 2;
            out[fill[t.v[r]]++] = {t.v[r], t.v[(r + 1) % 3], t.v[(r + 2) % 3]};
        }
        for (int i = 0; i < n_real_; ++i)
            if (start[i + 1] - start[i] > 1) std::sort(out.begin() + start[i], out.begin() + start[i + 1]);
        return out;
    }

private:
    // distance of (x, y) along the Hilbert curve of a 2^bits x 2^bits grid (x, y >= 0)
    static uint64_t hilbert(int bits, long long x, long long y) {
        uint64_t d = 0;
        for (long long s = 1ll << (bits - 1); s > 0; s >>= 1) {
            const long long rx = (x & s) ? 1 : 0, ry = (y & s) ? 1 : 0;
            d += static_cast<uint64_t>(s) * static_cast<uint64_t>(s) * static_cast<uint64_t>((3 * rx) ^ ry);
            if (ry == 0) {                               // rotate the quadrant
                if (rx == 1) { x = s - 1 - (x & (s - 1)); y = s - 1 - (y & (s - 1)); }
                std::swap(x, y);
            }
            x &= s - 1;
            y &= s - 1;
        }
        return d;
    }

    int locate(const Pt& q) const {
        int t = last_;
        if (t < 0 || !t_[t].alive) {
            for (t = static_cast<int>(t_.size()) - 1; t >= 0 && !t_[t].alive; --t) {}
        }
        for (size_t guard = 0; guard < 4 * t_.size() + 16; ++guard) {
            const Tri& T = t_[t];
            int next = -1;
            for (int e = 0; e < 3; ++e) {
                const Pt& a = p_[T.v[(e + 1) % 3]];
                const Pt& b = p_[T.v[(e + 2) % 3]];
                if (orient(a, b, q) < 0) { next = T.nb[e]; break; }
            }
            if (next < 0) return t;
            t = next;
        }
        // walk did not converge (cannot happen with exact predicates): fall back to a scan
        for (int k = 0; k < static_cast<int>(t_.size()); ++k) {
            if (!t_[k].alive) continue;
            const Tri& T = t_[k];
            if (orient(p_[T.v[0]], p_[T.v[1]], q) >= 0 && orient(p_[T.v[1]], p_[T.v[2]], q) >= 0 &&
                orient(p_[T.v[2]], p_[T.v[0]], q) >= 0)
                return k;
        }
        return 0;
    }

    int new_tri(int a, int b, int c) {
        Tri T{{a, b, c}, {-1, -1, -1}, true};
        if (!free_.empty()) {
            const int k = free_.back();
            free_.pop_back();
            t_[k] = T;
            return k;
        }
        t_.push_back(T);
        return static_cast<int>(t_.size()) - 1;
    }

    void insert(int pi) {
        const Pt& q = p_[pi];
        const int t0 = locate(q);
        // cavity: triangles whose circumcircle strictly contains q, connected to t0
        cavity_.clear();
        stack_.assign(1, t0);
        mark_.resize(t_.size(), 0);
        ++stamp_;
        if (stamp_ == 0) { std::fill(mark_.begin(), mark_.end(), 0u); stamp_ = 1; }
        mark_[t0] = stamp_;
        while (!stack_.empty()) {
            const int t = stack_.back();
            stack_.pop_back();
            cavity_.push_back(t);
            for (int e = 0; e < 3; ++e) {
                const int n = t_[t].nb[e];
                if (n < 0 || mark_[n] == stamp_) continue;
                const Tri& N = t_[n];
                if (incircle(p_[N.v[0]], p_[N.v[1]], p_[N.v[2]], q) > 0) {
                    mark_[n] = stamp_;
                    stack_.push_back(n);
                }
            }
        }
        // boundary edges (a, b) of the cavity, counter-clockwise as seen from inside
        edges_.clear();
        for (int t : cavity_) {
            const Tri T = t_[t];
            for (int e = 0; e < 3; ++e) {
                const int n = T.nb[e];
                if (n >= 0 && mark_[n] == stamp_) continue;
                int slot = -1;
                if (n >= 0)
                    for (int k = 0; k < 3; ++k) if (t_[n].nb[k] == t) slot = k;
                edges_.push_back({T.v[(e + 1) % 3], T.v[(e + 2) % 3], n, slot});
            }
        }
        for (int t : cavity_) { t_[t].alive = false; free_.push_back(t); }
        // fan from q; new triangle (a, b, q): nb[2] = outer, nb[0] = across (b, q), nb[1] = across (q, a)
        first_of_.clear();
        std::vector<int>& made = made_;
        made.clear();
        for (const BEdge& E : edges_) {
            const int k = new_tri(E.a, E.b, pi);
            if (static_cast<int>(mark_.size()) < static_cast<int>(t_.size())) mark_.resize(t_.size(), 0);
            t_[k].nb[2] = E.outer;
            if (E.outer >= 0) t_[E.outer].nb[E.outer_slot] = k;
            made.push_back(k);
        }
        // stitch the fan: triangle with edge starting at vertex a meets the one ending at a (the fan
        // is small -- ~6 triangles -- so a linear search beats sorting)
        const size_t nm = made.size();
        for (size_t i = 0; i < nm; ++i) {
            const int k = made[i];
            const int b = t_[k].v[1];
            for (size_t j = 0; j < nm; ++j) {
                const int m = made[j];
                if (t_[m].v[0] == b) {                   // triangle (b, c, q)
                    t_[k].nb[0] = m;                     // across (b, q)
                    t_[m].nb[1] = k;                     // across (q, b) of m
                    break;
                }
            }
        }
        last_ = made.empty() ? -1 : made.back();
    }

    struct BEdge { int a, b, outer, outer_slot; };
    std::vector<Pt> p_;
    std::vector<Tri> t_;
    std::vector<int> free_, cavity_, stack_, made_;
    std::vector<unsigned> mark_;
    unsigned stamp_ = 0;
    std::vector<BEdge> edges_;                    // cavity boundary of the current insertion
    std::vector<std::pair<int, int>> first_of_;
    int n_real_ = 0;
    int last_ = 0;
};

// Divide-and-conquer Delaunay (Guibas & Stolfi 1985, quad-edge subdivision) in Dwyer's form (1987): the points,
// sorted by x, are cut into vertical strips of about 2 sqrt(n) points; each strip is triangulated by the same
// divide and conquer with horizontal cuts (its points sorted by (y, -x): the frame turned by 90 degrees, which
// the orientation and in-circle predicates do not see), then the strips are merged along vertical seams.  Every
// merge walks only its seam (with vertical cuts alone the slabs are as tall as the image and each of the log n
// levels re-walks all of it: 39 ms for 38k points, slower than the incremental form).  Strips triangulate on up
// to 16 host threads, the top merges too.  Exact predicates as above (64-bit for coordinate differences below
// 2^14, 128-bit otherwise).  Co-circular points: any triangulation the merges settle on is Delaunay; it need not
// be the incremental one's (neither is cv::Subdiv2D's), and it does not depend on the thread
// count (the strips and split points are fixed by n).  The Hilbert-order incremental insertion stays the
// fallback (duplicate points, fewer than 3 points per strip, edge-pool overflow).
// The quad-edge arrays of one triangulation, kept between calls (DelaunayDC takes one from this pool and gives it
// back): fresh ones were ~10 MB of first-touch page faults per 68k-point call, 6 of its 57 ms on one host thread.
struct DcWorkspace {
    std::vector<int> onext, org, order;
    std::vector<unsigned char> alive;
};
std::mutex g_dc_mu;
std::vector<std::unique_ptr<DcWorkspace>> g_dc_free;

class DelaunayDC {
public:
    explicit DelaunayDC(const std::vector<Pt>& pts)
        : p_(pts), n_(static_cast<int>(pts.size())), ws_(take_ws()), onext_(ws_->onext), org_(ws_->org),
          order_(ws_->order), alive_(ws_->alive) {}
    ~DelaunayDC() {
        std::lock_guard<std::mutex> g(g_dc_mu);
        if (g_dc_free.size() < 8) g_dc_free.push_back(std::move(ws_));
    }
    DelaunayDC(const DelaunayDC&) = delete;
    DelaunayDC& operator=(const DelaunayDC&) = delete;

    // false: the incremental form must do it (duplicate points, degenerate strips, edge pool exhausted)
    bool run() {
        if (n_ < 3) return false;
        // (x, y) order: a counting sort on x keeps the input order within one x, which is y order for the
        // support points (strip-major, rows rising within a strip); anything else gets a comparison sort
        order_.resize(n_);
        long long xmin = p_[0].x, xmax = p_[0].x;
        for (const Pt& q : p_) { xmin = std::min(xmin, q.x); xmax = std::max(xmax, q.x); }
        auto xy_less = [&](int a, int b) { return p_[a].x != p_[b].x ? p_[a].x < p_[b].x : p_[a].y < p_[b].y; };
        if (xmax - xmin < 4 * static_cast<long long>(n_) + 65536) {
            std::vector<int> cnt(static_cast<size_t>(xmax - xmin) + 2, 0);
            for (const Pt& q : p_) ++cnt[q.x - xmin + 1];
            for (size_t k = 1; k < cnt.size(); ++k) cnt[k] += cnt[k - 1];
            for (int i = 0; i < n_; ++i) order_[cnt[p_[i].x - xmin]++] = i;
            bool sorted = true;
            for (int i = 1; i < n_ && sorted; ++i) sorted = !xy_less(order_[i], order_[i - 1]);
            if (!sorted) std::sort(order_.begin(), order_.end(), xy_less);
        } else {
            for (int i = 0; i < n_; ++i) order_[i] = i;
            std::sort(order_.begin(), order_.end(), xy_less);
        }
        for (int i = 1; i < n_; ++i)
            if (p_[order_[i]].x == p_[order_[i - 1]].x && p_[order_[i]].y == p_[order_[i - 1]].y) return false;
        // strips: a power of two, ~2 sqrt(n) points each, at least 8
        int S = 1;
        while (S * 2 <= static_cast<int>(std::sqrt(static_cast<double>(n_)) / 2.0) && n_ / (S * 2) >= 8) S *= 2;
        strip_lo_.resize(S + 1);
        for (int k = 0; k <= S; ++k) strip_lo_[k] = static_cast<int>(static_cast<long long>(n_) * k / S);
        strips_.assign(S, EdgePair{-1, -1});
        const unsigned hw = std::thread::hardware_concurrency();
        int T = (S > 1 && n_ >= 4096) ? static_cast<int>(std::min<unsigned>(std::min<unsigned>(hw ? hw : 1, 16u), S)) : 1;
        if (const char* e = std::getenv("ACMMP_DELAUNAY_THREADS")) T = std::max(1, std::min(T, std::atoi(e)));   // tests
        // quad pool: each strip thread a contiguous range (a strip of m points never holds more than 3m live
        // edges -- a planar subdivision -- and reuses its deleted ones), the merges the rest through one counter.
        // (One shared counter for everything interleaved the threads' quads: false sharing and a contended
        // atomic made the strips 10x slower.)
        size_t base = 0;
        for (int t = 0; t < T; ++t) {
            pool_[t].bump = base;
            for (int k = t; k < S; k += T) base += 3 * static_cast<size_t>(strip_lo_[k + 1] - strip_lo_[k]) + 16;
            pool_[t].end = base;
            base = (base + 15) & ~static_cast<size_t>(15);     // next thread's range on its own cache lines
        }
        merge_base_ = base;
        next_.store(base);
        cap_ = base + 3 * static_cast<size_t>(n_) + 1024;
        if (onext_.size() < 4 * cap_) onext_.resize(4 * cap_);   // (written before read: no clearing)
        if (org_.size() < 2 * cap_) org_.resize(2 * cap_);
        if (alive_.size() < cap_) alive_.resize(cap_);
        std::fill(alive_.begin(), alive_.begin() + static_cast<std::ptrdiff_t>(cap_), static_cast<unsigned char>(0));
        auto strip_task = [&](int t) {
            for (int k = t; k < S; k += T) {
                const int lo = strip_lo_[k], hi = strip_lo_[k + 1];
                std::sort(order_.begin() + lo, order_.begin() + hi, [&](int a, int b) {
                    return p_[a].y != p_[b].y ? p_[a].y < p_[b].y : p_[a].x > p_[b].x;
                });
                const EdgePair r = build(lo, hi, t);            // (y, -x) frame: edges out of its lowest / highest point
                strips_[k] = r.le < 0 ? EdgePair{-1, -1} : to_x_frame(r.le);
            }
        };
        HostPool::get().run(T, strip_task);
        for (TaskPool& tp : pool_) tp.bump = tp.end = 0;        // the merges allocate through next_
        for (const EdgePair& e : strips_)
            if (e.le < 0) return false;
        // merge the strips along vertical seams; the halves of the top levels on their own threads
        par_levels_ = 0;
        for (int t = T; t > 1 && (S >> par_levels_) > 1; t >>= 1) ++par_levels_;
        for (TaskPool& tp : pool_) tp.free.clear();
        const EdgePair r = merge_strips(0, S, 0, 0);
        return r.le >= 0 && !overflow_.load();
    }

    std::vector<std::array<int, 3>> triangles() const {
        // every face bounded by three edges and turning left: one triangle, kept from the directed edge leaving its
        // lowest point index a, in (a, b, c) order.  The live quads are scanned in parallel ranges; each triangle is
        // counted into its point a's bucket (atomics), the buckets' prefix taken, every triangle placed into its
        // bucket (atomic cursors, so any order within a bucket) and each bucket sorted -- in parallel throughout
        // (round 5 concatenated the ranges' lists and bucketed them with one serial counting sort: 15 of the 57 ms
        // of a 68k-point call on one host thread; walking each point's edge ring instead had the scan's locality
        // lost, +20 ms on one thread)
        const size_t used = std::min(next_.load(), cap_);      // (the strip ranges lie below merge_base_)
        const unsigned hw = std::thread::hardware_concurrency();
        const int T = used > 65536 ? static_cast<int>(std::min<unsigned>(hw ? hw : 1, 16u)) : 1;
        auto run_on = [&](auto&& f) { HostPool::get().run(T, f); };
        auto lo = [&](int t) { return static_cast<int>(static_cast<long long>(n_) * t / T); };
        std::vector<std::vector<std::array<int, 3>>> part(T);
        std::unique_ptr<std::atomic<int>[]> cnt(new std::atomic<int>[static_cast<size_t>(n_) + 1]);
        run_on([&](int t) {
            for (int a = lo(t); a < lo(t + 1); ++a) cnt[a + 1].store(0, std::memory_order_relaxed);
            if (t == 0) cnt[0].store(0, std::memory_order_relaxed);
        });
        run_on([&](int t) {
            std::vector<std::array<int, 3>>& out = part[t];
            out.reserve(used / T + 16);
            for (size_t q = used * t / T; q < used * (t + 1) / T; ++q) {
                if (!alive_[q]) continue;
                for (int r = 0; r < 4; r += 2) {
                    const int e = static_cast<int>(4 * q + r);
                    const int a = org(e), e1 = lnext(e), b = org(e1);
                    if (!(a < b)) continue;
                    const int e2 = lnext(e1), c = org(e2);
                    if (!(a < c) || lnext(e2) != e) continue;
                    if (orient(p_[a], p_[b], p_[c]) <= 0) continue;
                    out.push_back({a, b, c});
                    cnt[a + 1].fetch_add(1, std::memory_order_relaxed);
                }
            }
        });
        std::vector<int> start(static_cast<size_t>(n_) + 1);
        start[0] = 0;
        for (int i = 0; i < n_; ++i) start[i + 1] = start[i] + cnt[i + 1].load(std::memory_order_relaxed);
        run_on([&](int t) {                                    // the cursors: each bucket's start
            for (int a = lo(t); a < lo(t + 1); ++a) cnt[a].store(start[a], std::memory_order_relaxed);
        });
        std::vector<std::array<int, 3>> out(static_cast<size_t>(start[n_]));
        run_on([&](int t) {
            for (const auto& tr : part[t]) out[cnt[tr[0]].fetch_add(1, std::memory_order_relaxed)] = tr;
        });
        run_on([&](int t) {
            for (int a = lo(t); a < lo(t + 1); ++a)
                if (start[a + 1] - start[a] > 1) std::sort(out.begin() + start[a], out.begin() + start[a + 1]);
        });
        return out;
    }

private:
    struct EdgePair { int le, re; };
    // quad-edge navigation: edge e = 4 q + r, r the rotation
    static int rot(int e) { return (e & ~3) | ((e + 1) & 3); }
    static int sym(int e) { return (e & ~3) | ((e + 2) & 3); }
    static int rotinv(int e) { return (e & ~3) | ((e + 3) & 3); }
    int onext(int e) const { return onext_[e]; }
    int oprev(int e) const { return rot(onext_[rot(e)]); }
    int lnext(int e) const { return rot(onext_[rotinv(e)]); }
    int rprev(int e) const { return onext_[sym(e)]; }
    int org(int e) const { return org_[(e >> 2) * 2 + ((e & 3) >> 1)]; }
    int dest(int e) const { return org(sym(e)); }
    void set_org(int e, int v) { org_[(e >> 2) * 2 + ((e & 3) >> 1)] = v; }

    // -1 when the pool is exhausted (a planar subdivision of n points has < 3n edges, so 6n + 1024 quads hold
    // every task's live edges and free lists; the check keeps a bad input from writing out of bounds)
    int make_edge(int tid, int a, int b) {
        int q;
        std::vector<int>& fr = pool_[tid].free;
        if (!fr.empty()) { q = fr.back(); fr.pop_back(); }
        else if (pool_[tid].bump < pool_[tid].end) { q = static_cast<int>(pool_[tid].bump++); }
        else {
            const size_t k = next_.fetch_add(1);
            if (k >= cap_) { overflow_.store(true); return -1; }
            q = static_cast<int>(k);
        }
        const int e = 4 * q;
        onext_[e] = e; onext_[e + 2] = e + 2; onext_[e + 1] = e + 3; onext_[e + 3] = e + 1;
        set_org(e, a); set_org(e + 2, b);
        alive_[q] = 1;
        return e;
    }
    void splice(int a, int b) {
        const int al = rot(onext_[a]), be = rot(onext_[b]);
        std::swap(onext_[a], onext_[b]);
        std::swap(onext_[al], onext_[be]);
    }
    int connect(int tid, int a, int b) {
        const int e = make_edge(tid, dest(a), org(b));
        if (e < 0) return e;
        splice(e, lnext(a));
        splice(sym(e), b);
        return e;
    }
    void remove(int tid, int e) {
        splice(e, oprev(e));
        splice(sym(e), oprev(sym(e)));
        alive_[e >> 2] = 0;
        pool_[tid].free.push_back(e >> 2);
    }
    bool ccw(int a, int b, int c) const { return orient(p_[a], p_[b], p_[c]) > 0; }
    bool rightof(int x, int e) const { return ccw(x, dest(e), org(e)); }
    bool leftof(int x, int e) const { return ccw(x, org(e), dest(e)); }
    bool in_circle(int a, int b, int c, int d) const { return incircle(p_[a], p_[b], p_[c], p_[d]) > 0; }
    bool xless(int a, int b) const { return p_[a].x != p_[b].x ? p_[a].x < p_[b].x : p_[a].y < p_[b].y; }

    // A strip triangulated in the (y, -x) frame hands back the hull edge out of its first point with the outer
    // face on its right; walking the hull (sym . lnext . sym steps to the previous such edge) finds the (x, y)
    // frame's pair: the one out of the leftmost point, and the reverse of the one into the rightmost.
    EdgePair to_x_frame(int e0) const {
        int e = e0, le = -1, into_r = -1, vl = org(e0), vr = org(e0);
        size_t guard = 0;
        do {
            if (xless(org(e), vl) || org(e) == vl) { vl = org(e); le = e; }
            if (!xless(dest(e), vr)) { vr = dest(e); into_r = e; }
            e = sym(lnext(sym(e)));
        } while (e != e0 && ++guard < 4 * static_cast<size_t>(n_) + 16);
        if (le < 0 || into_r < 0) return {-1, -1};
        return {le, sym(into_r)};
    }

    // the Delaunay triangulation of order_[lo, hi) (sorted in the frame it is cut in): (le, re) = the
    // counter-clockwise hull edge out of its first point and the clockwise hull edge out of its last
    EdgePair build(int lo, int hi, int tid) {
        const int n = hi - lo;
        if (overflow_.load(std::memory_order_relaxed)) return {-1, -1};
        if (n == 2) {
            const int a = make_edge(tid, order_[lo], order_[lo + 1]);
            if (a < 0) return {-1, -1};
            return {a, sym(a)};
        }
        if (n == 3) {
            const int s1 = order_[lo], s2 = order_[lo + 1], s3 = order_[lo + 2];
            const int a = make_edge(tid, s1, s2);
            const int b = a < 0 ? -1 : make_edge(tid, s2, s3);
            if (b < 0) return {-1, -1};
            splice(sym(a), b);
            if (ccw(s1, s2, s3)) { if (connect(tid, b, a) < 0) return {-1, -1}; return {a, sym(b)}; }
            if (ccw(s1, s3, s2)) { const int c = connect(tid, b, a); if (c < 0) return {-1, -1}; return {sym(c), c}; }
            return {a, sym(b)};                              // collinear
        }
        const int mid = lo + n / 2;
        const EdgePair L = build(lo, mid, tid);
        const EdgePair R = build(mid, hi, tid);
        return merge(L, R, tid);
    }

    EdgePair merge_strips(int s0, int s1, int depth, int tid) {
        if (s1 - s0 == 1) return strips_[s0];
        const int mid = (s0 + s1) / 2;
        EdgePair L, R;
        if (depth < par_levels_) {
            // the right half on its own thread (free list tid_r), the left half on this one
            const int tid_r = tid + (1 << (par_levels_ - 1 - depth));
            HostPool::get().run(2, [&](int h) {
                if (h == 0) L = merge_strips(s0, mid, depth + 1, tid);
                else R = merge_strips(mid, s1, depth + 1, tid_r);
            });
            pool_[tid].free.insert(pool_[tid].free.end(), pool_[tid_r].free.begin(), pool_[tid_r].free.end());
            pool_[tid_r].free.clear();
        } else {
            L = merge_strips(s0, mid, depth + 1, tid);
            R = merge_strips(mid, s1, depth + 1, tid);
        }
        return merge(L, R, tid);
    }

    // the merge step of Guibas & Stolfi: L's points all precede R's in the cut's frame
    EdgePair merge(EdgePair L, EdgePair R, int tid) {
        if (L.le < 0 || R.le < 0 || overflow_.load()) return {-1, -1};
        int ldo = L.le, ldi = L.re, rdi = R.le, rdo = R.re;
        for (;;) {                                           // lower common tangent
            if (leftof(org(rdi), ldi)) ldi = lnext(ldi);
            else if (rightof(org(ldi), rdi)) rdi = rprev(rdi);
            else break;
        }
        int basel = connect(tid, sym(rdi), ldi);
        if (basel < 0) return {-1, -1};
        if (org(ldi) == org(ldo)) ldo = sym(basel);
        if (org(rdi) == org(rdo)) rdo = basel;
        for (;;) {                                           // the rising bubble
            int lcand = onext(sym(basel));
            if (rightof(dest(lcand), basel)) {
                while (in_circle(dest(basel), org(basel), dest(lcand), dest(onext(lcand)))) {
                    const int t = onext(lcand);
                    remove(tid, lcand);
                    lcand = t;
                }
            }
            int rcand = oprev(basel);
            if (rightof(dest(rcand), basel)) {
                while (in_circle(dest(basel), org(basel), dest(rcand), dest(oprev(rcand)))) {
                    const int t = oprev(rcand);
                    remove(tid, rcand);
                    rcand = t;
                }
            }
            const bool lval = rightof(dest(lcand), basel), rval = rightof(dest(rcand), basel);
            if (!lval && !rval) break;
            if (!lval || (rval && in_circle(dest(lcand), org(lcand), org(rcand), dest(rcand))))
                basel = connect(tid, rcand, sym(basel));
            else
                basel = connect(tid, sym(basel), sym(lcand));
            if (basel < 0) return {-1, -1};
        }
        return {ldo, rdo};
    }

    static std::unique_ptr<DcWorkspace> take_ws() {
        std::lock_guard<std::mutex> g(g_dc_mu);
        if (g_dc_free.empty()) return std::make_unique<DcWorkspace>();
        std::unique_ptr<DcWorkspace> w = std::move(g_dc_free.back());
        g_dc_free.pop_back();
        return w;
    }
    const std::vector<Pt>& p_;
    int n_;
    std::unique_ptr<DcWorkspace> ws_;
    std::vector<int>& onext_;
    std::vector<int>& org_;
    std::vector<int>& order_;
    std::vector<unsigned char>& alive_;
    size_t cap_ = 0;
    std::vector<int> strip_lo_;
    std::vector<EdgePair> strips_;
    std::atomic<size_t> next_{0};
    std::atomic<bool> overflow_{false};
    // per task: its free quads and its pool range, each on its own cache lines (adjacent, every make_edge of one
    // thread invalidated the others' lines)
    struct alignas(128) TaskPool {
        std::vector<int> free;
        size_t bump = 0, end = 0;
    };
    TaskPool pool_[16];
    size_t merge_base_ = 0;
    int par_levels_ = 0;
};

// DelaunayTriangulation's triangles (ACMMP.cpp:932-955) in triangles()' order: the divide-and-conquer form, or
// the incremental one when that declines
std::vector<std::array<int, 3>> delaunay_triangles(const std::vector<Pt>& pts, long long extent) {
    if (!std::getenv("ACMMP_DELAUNAY_INCREMENTAL")) {
        DelaunayDC dc(pts);
        if (dc.run()) return dc.triangles();
    }
    Delaunay d(pts, extent);
    d.run();
    return d.triangles();
}

// Get3DPointonRefCam (ACMMP.cpp:287-312), float maths with the reference's promotions
void point_on_ref_cam(int x, int y, float depth, const acmmp_camera& c, float out[3]) {
    if (c.model == ACMMP_SPHERE) {
        const float lon = static_cast<float>((static_cast<float>(x) - c.params[1]) / static_cast<float>(c.width) *
                                             2.0f * kMPi);
        const float lat = static_cast<float>(-(static_cast<float>(y) - c.params[2]) /
                                             static_cast<float>(c.height) * kMPi);
        out[0] = std::cos(lat) * std::sin(lon) * depth;
        out[1] = -std::sin(lat) * depth;
        out[2] = std::cos(lat) * std::cos(lon) * depth;
    } else {
        out[0] = depth * (static_cast<float>(x) - c.K[2]) / c.K[0];
        out[1] = depth * (static_cast<float>(y) - c.K[5]) / c.K[4];
        out[2] = depth;
    }
}

// Run f(0..n-1) on the host's cores (at most 16 threads); order of completion is irrelevant to
// every caller (each writes disjoint cells or combines with an order-independent max).
template <typename F>
void parallel_for(int n, F&& f) {
    const unsigned hw = std::thread::hardware_concurrency();
    const int nt = static_cast<int>(std::min<unsigned>(hw ? hw : 1, 16u));
    if (nt <= 1 || n < 256) {
        for (int i = 0; i < n; ++i) f(i);
        return;
    }
    std::atomic<int> next(0);
    auto worker = [&]() {
        for (;;) {
            const int b = next.fetch_add(64);
            if (b >= n) return;
            const int e = std::min(n, b + 64);
            for (int i = b; i < e; ++i) f(i);
        }
    };
    HostPool::get().run(nt, [&](int) { worker(); });
}

// GetSupportPoints (ACMMP.cpp:904-929): per 5x5 block in column-major block order, the first
// minimum-cost pixel of the block scanned column by column (strict '>' keeps the first), kept when
// its cost is < 0.1.  Column strips run in parallel into their own lists, concatenated in strip
// order -- the reference's point order, which the Delaunay insertion order depends on.
std::vector<int> support_points(const float* costs, int W, int H) {
    const int step = 5;
    const int strips = (W + step - 1) / step;
    std::vector<std::vector<int>> per(strips);
    parallel_for(strips, [&](int s) {
        const int col = s * step;
        const int cb = std::min(W, col + step);
        std::vector<int>& out = per[s];
        for (int row = 0; row < H; row += step) {
            float min_cost = 2.0f;
            int tx = 0, ty = 0;
            const int rb = std::min(H, row + step);
            for (int c = col; c < cb; ++c)
                for (int r = row; r < rb; ++r) {
                    const float v = costs[static_cast<size_t>(r) * W + c];
                    if (v < 2.0f && min_cost > v) { tx = c; ty = r; min_cost = v; }
                }
            if (min_cost < 0.1f) { out.push_back(tx); out.push_back(ty); }
        }
    });
    std::vector<int> all;
    for (const auto& v : per) all.insert(all.end(), v.begin(), v.end());
    return all;
}

// GetDepthFromPlaneParam's SPHERE ray (ACMMP.cpp:993-1006) is separable: sin/cos of the latitude
// depend on the row only and of the longitude on the column only, so a whole-image pass computes
// them once per row / column -- the same float values the per-pixel expressions give.
struct SphereTrig { float s, c; };
SphereTrig sphere_row(const acmmp_camera& c, int y) {
    const float lat = static_cast<float>(-(static_cast<float>(y) - c.params[2]) / static_cast<float>(c.height) * kMPi);
    return {std::sin(lat), std::cos(lat)};
}
SphereTrig sphere_col(const acmmp_camera& c, int x) {
    const float lon = static_cast<float>((static_cast<float>(x) - c.params[1]) / static_cast<float>(c.width) *
                                         2.0f * kMPi);
    return {std::sin(lon), std::cos(lon)};
}
float sphere_depth(const float plane[4], SphereTrig lat, SphereTrig lon) {
    const float dx = lat.c * lon.s, dy = -lat.s, dz = lat.c * lon.c;
    const float denom = plane[0] * dx + plane[1] * dy + plane[2] * dz;
    return (std::abs(denom) < 1e-6f) ? 1e6f : (-plane[3] / denom);
}

// GetPriorPlaneParams (ACMMP.cpp:957-989) through the three vertices' depths d3
// GetPriorPlaneParams on the points X[3] (Get3DPointonRefCam of the triangle's vertices)
void plane_through(float X[3][3], float plane[4]);

void prior_plane(const acmmp_camera& cam, const int tri_xy[6], const float d3[3], float plane[4]) {
    float X[3][3];
    for (int k = 0; k < 3; ++k) point_on_ref_cam(tri_xy[2 * k], tri_xy[2 * k + 1], d3[k], cam, X[k]);
    plane_through(X, plane);
}

// The same with a SPHERE camera's (sin, cos) of each row's latitude and each column's longitude from tables
// (sphere_row / sphere_col: the values point_on_ref_cam computes, so the same bits) instead of four libm calls
// per vertex -- those were most of the host half's plane fits (136k triangles at 2000x1500)
void prior_plane_trig(const int tri_xy[6], const float d3[3], const float2* row_trig, const float2* col_trig,
                      float plane[4]) {
    float X[3][3];
    for (int k = 0; k < 3; ++k) {
        const float2 lon = col_trig[tri_xy[2 * k]], lat = row_trig[tri_xy[2 * k + 1]];
        X[k][0] = lat.y * lon.x * d3[k];
        X[k][1] = -lat.x * d3[k];
        X[k][2] = lat.y * lon.y * d3[k];
    }
    plane_through(X, plane);
}

void plane_through(float X[3][3], float plane[4]) {

    // cv::SVD::solveZ on [X_k 1] (3x4): the null vector, i.e. the plane through the three points
    // (ACMMP.cpp:960-980).  Closed form: n = (X2-X1) x (X3-X1), w = -n.X1.
    const float e1[3] = {X[1][0] - X[0][0], X[1][1] - X[0][1], X[1][2] - X[0][2]};
    const float e2[3] = {X[2][0] - X[0][0], X[2][1] - X[0][1], X[2][2] - X[0][2]};
    float n4[4] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0], 0.f};
    n4[3] = -(n4[0] * X[0][0] + n4[1] * X[0][1] + n4[2] * X[0][2]);
    // ACMMP.cpp:981-988: normalise by the normal's length, sign so that w >= 0
    // std::pow(float, 2) is the double pow of the promoted value: its square, exact in double
    const double nx = n4[0], ny = n4[1], nz = n4[2];
    float norm2 = static_cast<float>(std::sqrt(nx * nx + ny * ny + nz * nz));
    if (n4[3] < 0) norm2 *= -1;
    for (int k = 0; k < 4; ++k) plane[k] = n4[k] / norm2;
}

}  // namespace

extern "C" {

acmmp_status acmmp_support_points(const float* costs, int W, int H, int* xy, int cap, int* n_out) {
    if (!costs || !n_out || W <= 0 || H <= 0 || cap < 0 || (cap > 0 && !xy)) return ACMMP_ERR_INVALID_ARGUMENT;
    const std::vector<int> pts = support_points(costs, W, H);
    const int n = static_cast<int>(pts.size() / 2);
    if (xy && cap > 0) std::memcpy(xy, pts.data(), sizeof(int) * 2 * static_cast<size_t>(std::min(n, cap)));
    *n_out = n;
    return n <= cap ? ACMMP_OK : ACMMP_ERR_INVALID_ARGUMENT;
}

acmmp_status acmmp_delaunay(const int* xy, int n, int W, int H, int* tri_xy, int cap, int* n_tri) {
    if (!n_tri || n < 0 || (n > 0 && !xy) || cap < 0 || (cap > 0 && !tri_xy)) return ACMMP_ERR_INVALID_ARGUMENT;
    *n_tri = 0;
    if (n == 0) return ACMMP_OK;                           // ACMMP.cpp:934-936
    std::vector<Pt> pts(n);
    for (int i = 0; i < n; ++i) pts[i] = {xy[2 * i], xy[2 * i + 1]};
    const auto tris = delaunay_triangles(pts, std::max<long long>(std::max(W, H), 1));
    const int m = static_cast<int>(tris.size());
    for (int k = 0; k < std::min(m, cap); ++k)
        for (int j = 0; j < 3; ++j) {
            tri_xy[6 * k + 2 * j] = xy[2 * tris[k][j]];
            tri_xy[6 * k + 2 * j + 1] = xy[2 * tris[k][j] + 1];
        }
    *n_tri = m;
    return m <= cap ? ACMMP_OK : ACMMP_ERR_INVALID_ARGUMENT;
}

acmmp_status acmmp_prior_plane_params(const acmmp_camera* cam, const float* depths, int W, int H, const int tri_xy[6],
                                      float plane[4]) {
    if (!cam || !depths || !tri_xy || !plane || W <= 0 || H <= 0) return ACMMP_ERR_INVALID_ARGUMENT;
    float d3[3];
    for (int k = 0; k < 3; ++k) {
        const int x = tri_xy[2 * k], y = tri_xy[2 * k + 1];
        if (x < 0 || x >= W || y < 0 || y >= H) return ACMMP_ERR_INVALID_ARGUMENT;
        d3[k] = depths[static_cast<size_t>(y) * W + x];
    }
    prior_plane(*cam, tri_xy, d3, plane);
    return ACMMP_OK;
}

float acmmp_depth_from_plane_param(const acmmp_camera* cam, const float plane[4], int x, int y) {
    const acmmp_camera& c = *cam;
    if (c.model == ACMMP_SPHERE) {                          // ACMMP.cpp:993-1006
        const SphereTrig r = sphere_row(c, y), k = sphere_col(c, x);
        return sphere_depth(plane, r, k);
    }
    // ACMMP.cpp:1008-1009 (int x - float K[2] -> float)
    return -plane[3] * c.K[0] /
           ((x - c.K[2]) * plane[0] + (c.K[0] / c.K[4]) * (y - c.K[5]) * plane[1] + c.K[0] * plane[2]);
}

acmmp_status acmmp_planar_prior_host(const acmmp_camera* cam, const float* depths, const float* costs, int W, int H,
                                     float depth_min, float depth_max, float* prior_planes, uint32_t* masks,
                                     int* n_triangles) {
    if (!cam || !depths || !costs || !prior_planes || !masks || W <= 0 || H <= 0) return ACMMP_ERR_INVALID_ARGUMENT;
    const size_t P = static_cast<size_t>(W) * H;
    acmmp::PlanarTriangles pt;
    const acmmp_status st = acmmp::planar_triangles(*cam, depths, costs, W, H, &pt);
    if (st != ACMMP_OK) return st;
    const int m = static_cast<int>(pt.step.size());
    // Rasterise in parallel.  The reference overwrites labels in triangle order, so a pixel ends with
    // the label of the LAST triangle that covered it -- the largest label: an atomic max gives the same
    // mask whatever the thread schedule.
    std::vector<uint32_t> lab(P, 0u);
    parallel_for(m, [&](int k) {
        const uint32_t label = static_cast<uint32_t>(k) + 1u;
        const int* t = &pt.tri[6 * static_cast<size_t>(k)];
        const float step = pt.step[k];
        for (float p = 0; p < 1.0; p += step) {
            for (float q = 0; q < 1.0 - p; q += step) {
                const int x = static_cast<int>(static_cast<double>(p * t[0] + q * t[2]) + (1.0 - p - q) * t[4]);
                const int y = static_cast<int>(static_cast<double>(p * t[1] + q * t[3]) + (1.0 - p - q) * t[5]);
                uint32_t* cell = &lab[static_cast<size_t>(y) * W + x];
                uint32_t cur = __atomic_load_n(cell, __ATOMIC_RELAXED);
                while (cur < label && !__atomic_compare_exchange_n(cell, &cur, label, true, __ATOMIC_RELAXED,
                                                                  __ATOMIC_RELAXED)) {}
            }
        }
    });
    // prior depth range check (main.cpp:167-180) and CudaPlanarPriorInitialization (ACMMP.cpp:851-861);
    // every pixel is independent (mask_tri holds float labels idx + 1.0, exact below 2^24)
    const bool sphere = cam->model == ACMMP_SPHERE;
    parallel_for(H, [&](int j) {
        const SphereTrig lat = sphere ? SphereTrig{pt.row_trig[j].x, pt.row_trig[j].y} : SphereTrig{0.f, 0.f};
        for (int i = 0; i < W; ++i) {
            const size_t c = static_cast<size_t>(j) * W + i;
            uint32_t l = lab[c];
            if (l > 0) {
                const float* pl = &pt.plane[4 * static_cast<size_t>(l - 1)];
                const float d = sphere ? sphere_depth(pl, lat, SphereTrig{pt.col_trig[i].x, pt.col_trig[i].y})
                                       : acmmp_depth_from_plane_param(cam, pl, i, j);
                if (!(d <= depth_max && d >= depth_min)) l = 0;
            }
            masks[c] = l;
            if (l > 0) std::memcpy(prior_planes + 4 * c, &pt.plane[4 * static_cast<size_t>(l - 1)], 4 * sizeof(float));
            else std::memset(prior_planes + 4 * c, 0, 4 * sizeof(float));
        }
    });
    if (n_triangles) *n_triangles = m;
    return ACMMP_OK;
}

}  // extern "C"

namespace acmmp {

// Host half of the planar block (planar.h): GetSupportPoints + DelaunayTriangulation, the triangles
// ProcessProblem labels (main.cpp:138-145: all vertices inside the image, labels 1, 2, ... in
// triangle order), each one's plane (GetPriorPlaneParams through the first run's depths) and
// sampling step, the per-triangle count of the p loop (main.cpp:153) as a prefix, and the SPHERE
// row/column trig tables of GetDepthFromPlaneParam.
acmmp_status planar_triangles(const acmmp_camera& cam, const float* depths, const float* costs, int W, int H,
                              PlanarTriangles* out) {
    const std::vector<int> xy = support_points(costs, W, H);
    std::vector<float> depth_at(xy.size() / 2);
    for (size_t i = 0; i < depth_at.size(); ++i)
        depth_at[i] = depths[static_cast<size_t>(xy[2 * i + 1]) * W + xy[2 * i]];
    return planar_triangles_pts(cam, xy, depth_at, W, H, out);
}

acmmp_status planar_triangles_pts(const acmmp_camera& cam, const std::vector<int>& xy,
                                  const std::vector<float>& depth_at, int W, int H, PlanarTriangles* out) {
    const int n = static_cast<int>(xy.size() / 2);
    std::vector<int> tri, tri_pt;                          // vertex coordinates / point indices
    const auto t0 = std::chrono::steady_clock::now();
    if (n > 0) {                                           // triangulate once (ACMMP.cpp:932-955)
        std::vector<Pt> pts(n);
        for (int i = 0; i < n; ++i) pts[i] = {xy[2 * i], xy[2 * i + 1]};
        const auto dt = delaunay_triangles(pts, std::max<long long>(std::max(W, H), 1));
        out->delaunay_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
        bool all_inside = true;                             // (support points always are: then no triangle drops out)
        for (int i = 0; i < n && all_inside; ++i)
            all_inside = xy[2 * i] >= 0 && xy[2 * i] < W && xy[2 * i + 1] >= 0 && xy[2 * i + 1] < H;
        if (all_inside) {
            tri.resize(6 * dt.size());
            tri_pt.resize(3 * dt.size());
            parallel_for(static_cast<int>(dt.size()), [&](int k) {
                for (int j = 0; j < 3; ++j) {
                    tri[6 * static_cast<size_t>(k) + 2 * j] = xy[2 * dt[k][j]];
                    tri[6 * static_cast<size_t>(k) + 2 * j + 1] = xy[2 * dt[k][j] + 1];
                    tri_pt[3 * static_cast<size_t>(k) + j] = dt[k][j];
                }
            });
        } else {
            for (const auto& t : dt) {
                bool inside = true;
                for (int j = 0; j < 3; ++j) {
                    const int x = xy[2 * t[j]], y = xy[2 * t[j] + 1];
                    inside = inside && x >= 0 && x < W && y >= 0 && y < H;
                }
                if (!inside) continue;
                for (int j = 0; j < 3; ++j) {
                    tri.push_back(xy[2 * t[j]]);
                    tri.push_back(xy[2 * t[j] + 1]);
                    tri_pt.push_back(t[j]);
                }
            }
        }
    }
    const int m = static_cast<int>(tri.size() / 6);
    out->tri = std::move(tri);
    out->plane.assign(4 * static_cast<size_t>(m), 0.f);
    out->step.assign(m, 0.f);
    out->row_trig.clear();
    out->col_trig.clear();
    const bool sphere = cam.model == ACMMP_SPHERE;
    if (sphere) {
        out->row_trig.resize(H);
        out->col_trig.resize(W);
        for (int y = 0; y < H; ++y) { const SphereTrig r = sphere_row(cam, y); out->row_trig[y] = make_float2(r.s, r.c); }
        for (int x = 0; x < W; ++x) { const SphereTrig k = sphere_col(cam, x); out->col_trig[x] = make_float2(k.s, k.c); }
    }
    std::vector<long long> np(m, 0);
    parallel_for(m, [&](int k) {
        const int* t = &out->tri[6 * static_cast<size_t>(k)];
        // main.cpp:146-148's sqrt(pow(d, 2) + ...) in double: pow(d, 2) of an integer d is d * d exactly
        auto sq = [](int d) { return static_cast<double>(d) * static_cast<double>(d); };
        const float L01 = static_cast<float>(std::sqrt(sq(t[0] - t[2]) + sq(t[1] - t[3])));
        const float L02 = static_cast<float>(std::sqrt(sq(t[0] - t[4]) + sq(t[1] - t[5])));
        const float L12 = static_cast<float>(std::sqrt(sq(t[2] - t[4]) + sq(t[3] - t[5])));
        const float max_edge_length = std::max(L01, std::max(L02, L12));
        const float step = static_cast<float>(1.0 / max_edge_length);
        out->step[k] = step;
        long long c = 0;
        for (float p = 0; p < 1.0; p += step) ++c;
        np[k] = c;
        const float d3[3] = {depth_at[tri_pt[3 * k]], depth_at[tri_pt[3 * k + 1]], depth_at[tri_pt[3 * k + 2]]};
        if (sphere) prior_plane_trig(t, d3, out->row_trig.data(), out->col_trig.data(), &out->plane[4 * static_cast<size_t>(k)]);
        else prior_plane(cam, t, d3, &out->plane[4 * static_cast<size_t>(k)]);
    });
    out->first.assign(static_cast<size_t>(m) + 1, 0);
    for (int k = 0; k < m; ++k) out->first[k + 1] = out->first[k] + np[k];
    return ACMMP_OK;
}

}  // namespace acmmp
