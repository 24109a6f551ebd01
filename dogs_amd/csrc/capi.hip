// capi.hip -- extern "C" entry points of libdogs_hip.so (declared in include/dogs_hip.h).
//
// Owns the host-side orchestration of Rasterizer::forward/backward (rasterizer_impl.cu:334-676):
// carving of the private state blocks, the single host sync (instance count), launch order.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>
#include <map>
#include <tuple>
#include <chrono>
#include <mutex>
#include <atomic>
#include <thread>
#include <algorithm>
#include <atomic>
#include <thread>
#include <algorithm>

#include "../../include/dogs_hip.h"
#include "aux_kernels.h"
#include "blocksplit.h"
#include "optim.h"
#include "mask_conv.h"
#include "export.h"
#include "raster.h"
#include "sortscan.h"

namespace {

thread_local std::string g_err;

int fail(const char* fmt, const char* a = "", int b = 0) {
    char buf[512];
    snprintf(buf, sizeof(buf), fmt, a, b);
    g_err = buf;
    return 1;
}

#define HIP_OK(x)                                                                \
    do {                                                                         \
        hipError_t _e = (x);                                                     \
        if (_e != hipSuccess) return fail("HIP error: %s (line %d)", hipGetErrorString(_e), __LINE__); \
    } while (0)

#define DBG_SYNC(dbg, s)                                                         \
    do {                                                                         \
        if (dbg) {                                                               \
            HIP_OK(hipStreamSynchronize(s));                                     \
            HIP_OK(hipGetLastError());                                           \
        }                                                                        \
    } while (0)

// ---- optional per-kernel event profiling (dg_profile_*): brackets each launch with hipEvents on the
// caller's stream; used by bench.py for the live roofline figure.  Off by default (no events recorded).
struct ProfRec { const char* name; hipEvent_t a, b; };
bool g_prof = false;
std::vector<ProfRec> g_prof_recs;
std::vector<hipEvent_t> g_ev_pool;
hipEvent_t prof_event() {
    if (!g_ev_pool.empty()) { hipEvent_t e = g_ev_pool.back(); g_ev_pool.pop_back(); return e; }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
}
struct ProfScope {
    ProfRec r;
    hipStream_t s;
    bool on;
    ProfScope(const char* name, hipStream_t st) : s(st), on(g_prof) {
        if (on) { r.name = name; r.a = prof_event(); r.b = prof_event(); (void)hipEventRecord(r.a, s); }
    }
    ~ProfScope() {
        if (on) { (void)hipEventRecord(r.b, s); g_prof_recs.push_back(r); }
    }
};
#define PROF(name) ProfScope _prof_scope_##__LINE__(name, s)

constexpr size_t ALIGN = 256;
inline size_t al(size_t x) { return (x + ALIGN - 1) & ~(ALIGN - 1); }

struct Carver {
    char* base;
    size_t off = 0;
    explicit Carver(void* b) : base((char*)b) {}
    template <typename T>
    T* take(size_t count) {
        T* p = base ? (T*)(base + off) : nullptr;
        off += al(count * sizeof(T) + (count == 0 ? 1 : 0));
        return p;
    }
};

inline int tiles_x_of(int W) { return (W + 15) / 16; }
inline int tiles_y_of(int H) { return (H + 15) / 16; }
inline int unf_rw_of(int tiles_x) { return (tiles_x + 63) / 64; }  // bitmask words per tile row
#ifdef DG_PHASE2_SAT  // A/B switch: phase-2 membership from a summed-area table (two launches per view)
constexpr bool UNF_ROWS = false;
#else
constexpr bool UNF_ROWS = true;
#endif

struct Geom {
    uint32_t* counters;  // CNT_* (raster.h)
    float4* sp;  // 2 per Gaussian (raster.h)
    float4* rgbi;
    uint32_t *dkey, *cnt, *first_e;  // depth key, tile-rect area, first instance
    uint32_t* rcnt;                  // instances (= records of the backward) per Gaussian
    uint32_t* hist;                  // [DH_BINS] depth histogram of the prefix cut
    uint32_t* wtot;                  // [bin_waves(P)] per-wave instance totals of the binning walk
    uint64_t* wmask;                 // [bin_waves(P)] per-wave member ballot of the binning walk
    uint64_t* kmask;                 // [bin_waves(P) * KM_STEPS] kept ballots of the phase-1 count walk's first steps
    uint32_t* mlist;                 // [P] member lists of the fat binning waves
    void* scan_tmp;
    size_t bytes;
};
Geom carve_geom(void* base, int P) {
    Carver c(base);
    Geom g;
    const size_t n = (size_t)(P > 0 ? P : 1);
    g.counters = c.take<uint32_t>(16);
    g.sp = c.take<float4>(2 * n);
    g.rgbi = c.take<float4>(n);
    g.dkey = c.take<uint32_t>(n);
    g.cnt = c.take<uint32_t>(n);
    g.first_e = c.take<uint32_t>(n);
    g.rcnt = c.take<uint32_t>(n);
    g.hist = c.take<uint32_t>(gs::DH_BINS);
    g.wtot = c.take<uint32_t>((size_t)gs::bin_waves(P > 0 ? P : 1));
    g.wmask = c.take<uint64_t>((size_t)gs::bin_waves(P > 0 ? P : 1));
    g.kmask = c.take<uint64_t>((size_t)gs::bin_waves(P > 0 ? P : 1) * gs::KM_STEPS);
    g.mlist = c.take<uint32_t>(n);
    g.scan_tmp = c.take<char>(gs::bin_scan_temp_bytes(P > 0 ? P : 1));
    g.bytes = c.off;
    return g;
}

struct Image {
    float *final_T, *img_color, *img_invd;
    uint32_t *n_contrib, *max_contrib;
    uint2* ranges;
    uint2* ranges2;         // phase-2 lists of unfinished tiles
    uint8_t* unfinished;    // [T]
    float4* resume;         // [HW] raw colour + live threshold of unfinished tiles' pixels
    uint32_t* sat;          // [(ty+1)*(tx+1)] summed-area table of `unfinished`
    uint32_t* long_tiles;   // [T] queue of the long-list tile depth sort
    uint32_t *tile_cnt, *tile_cnt2;  // [T] per-tile instance counters of the phase-1 / phase-2 binning
    uint32_t* ohist;        // [2 ORDER_NB] the phase-2 launches' replay-order buckets (after tile_cnt2)
    uint32_t* order;        // [T] the backward's replay order (written by the phase-2 emission when phase 2 ran)
    uint32_t* unf_list;     // [T] the unfinished tiles, in the order phase 1 found them
    uint32_t* unf_sorted;   // [T] those with phase-2 instances, longest list first (the phase-2 emission)
    size_t bytes;
};
Image carve_image(void* base, int W, int H) {
    Carver c(base);
    Image im;
    const size_t HW = (size_t)W * H > 0 ? (size_t)W * H : 1;
    const size_t T = (size_t)tiles_x_of(W) * tiles_y_of(H) > 0 ? (size_t)tiles_x_of(W) * tiles_y_of(H) : 1;
    im.final_T = c.take<float>(HW);
    im.n_contrib = c.take<uint32_t>(HW);
    im.img_color = c.take<float>(3 * HW);
    im.img_invd = c.take<float>(HW);
    im.ranges = c.take<uint2>(T);
    im.max_contrib = c.take<uint32_t>(T);
    im.ranges2 = c.take<uint2>(T);
    im.unfinished = c.take<uint8_t>(T);
    im.resume = c.take<float4>(HW);
    {  // the SAT of the A/B build, or the phase-2 row bitmasks (u64: rows, column OR, row summary)
        const size_t txs = (size_t)tiles_x_of(W), tys = (size_t)tiles_y_of(H);
        const size_t sat_n = (txs + 1) * (tys + 1), rows_n = 2 * ((tys + 1) * ((txs + 63) / 64) + (tys + 63) / 64);
        im.sat = c.take<uint32_t>(sat_n > rows_n ? sat_n : rows_n);
    }
    im.long_tiles = c.take<uint32_t>(T);
    im.tile_cnt = c.take<uint32_t>(T);
    im.tile_cnt2 = c.take<uint32_t>(T + 2 * gs::ORDER_NB);  // + the replay-order histogram (zeroed by k_depth_cut)
    im.ohist = im.tile_cnt2 + T;
    im.order = c.take<uint32_t>(T);
    im.unf_list = c.take<uint32_t>(T);
    im.unf_sorted = c.take<uint32_t>(T);
    im.bytes = c.off;
    return im;
}

// Per-instance arrays of one binning phase; instances are indexed by emission order.
struct Binning {
    uint32_t* se;      // instances binned by tile, each tile in (depth, index) order
    uint32_t* se_tmp;  // scratch values of the long-list depth sort
    uint32_t* eg;      // Gaussian of each instance
    uint32_t* ik;      // depth key of each instance
    uint32_t *dk, *dk2;  // scratch keys of the long-list depth sort
    uint8_t* flag;     // the backward's record-written flag of each instance (zeroed by the emission)
    size_t bytes;
};
Binning carve_binning(void* base, int64_t K) {
    Carver c(base);
    Binning b;
    const size_t n = (size_t)(K > 0 ? K : 1);
    b.se = c.take<uint32_t>(n);
    b.se_tmp = c.take<uint32_t>(n);
    b.eg = c.take<uint32_t>(n);
    b.ik = c.take<uint32_t>(n);
    b.dk = c.take<uint32_t>(n);
    b.dk2 = c.take<uint32_t>(n);
    b.flag = c.take<uint8_t>(n);
    b.bytes = c.off;
    return b;
}
gs::BinArgs bin_args(const dg_raster_args* r, const Geom& g, const Image& im, int T, uint32_t cap, const Binning& b,
                     uint32_t* tile_cnt, uint2* ranges) {
    gs::BinArgs a;
    const int P = r->P, tx = tiles_x_of(r->W);
    a.D = (r->sh && r->M > 0) ? r->D : 0; a.M = r->M; a.means3D = r->means3D; a.campos = r->campos; a.dc = r->dc;
    a.sh = (r->sh && r->M > 0) ? r->sh : nullptr; a.colors = r->colors; a.rgbi = g.rgbi;
    a.P = P; a.tiles_x = tx; a.num_tiles = T; a.dkey = g.dkey; a.sp = g.sp; a.counters = g.counters;
    a.unf = im.unfinished; a.sat = im.sat; a.wtot = g.wtot; a.wmask = g.wmask; a.mlist = g.mlist; a.cap = cap; a.first_e = g.first_e; a.rcnt = g.rcnt;
    a.eg = b.eg; a.ikey = b.ik; a.flag = b.flag; a.tile_cnt = tile_cnt; a.ranges = ranges; a.s_e = b.se;
    a.unf_rows = nullptr; a.unf_rw = 0; a.unf_th = 0; a.probe = nullptr; a.colors_later = 0;
    a.ohist = nullptr; a.max_contrib = nullptr; a.ranges1 = nullptr; a.unf_list = nullptr; a.unf_sorted = nullptr;
    a.kmask = g.kmask;
    return a;
}
// per-tile (depth, index) order of a phase's binned lists
gs::DSortArgs dsort_args(const Binning& b, int64_t cap, int T, uint2* ranges, const uint8_t* only,
                         const uint32_t* gate, uint32_t* long_list, uint32_t* long_cnt) {
    gs::DSortArgs d;
    d.num_tiles = T; d.ranges = ranges; d.s_e = b.se; d.s_tmp = b.se_tmp; d.k_a = b.dk; d.k_b = b.dk2;
    d.ikey = b.ik; d.eg = b.eg; d.n_inst = (uint32_t)(cap > 0 ? cap : 1); d.only = only; d.gate = gate;
    d.long_list = long_list; d.long_cnt = long_cnt;
    return d;
}
#ifdef DG_NO_FUSED_SORT  // A/B switch: the phase-1 depth sort as its own launches
constexpr bool FUSED_SORT = false;
#else
constexpr bool FUSED_SORT = true;
#endif

// Pinned landing buffer + event for the forward's early counter read, one per calling thread while it lives: a
// thread's slot goes back to a process-wide pool when the thread exits (ADMM worker and RPC threads come and go), so
// the pinned buffers and events are bounded by the number of threads alive at once.
struct HostCounters {
    uint32_t* buf = nullptr;  // [0, 16) the counters, [16] the sequence word of the polled path
    uint32_t* dev = nullptr;  // buf as the device addresses it (null: copy with hipMemcpyAsync + event instead)
    hipEvent_t ev = nullptr;
    uint32_t seq = 0;
};
// The pool and its mutex are allocated once and never freed: a thread that exits during interpreter teardown (after
// the static destructors ran) still finds them alive.
std::mutex& hc_mu() { static auto* m = new std::mutex; return *m; }
std::vector<HostCounters>& hc_pool() { static auto* v = new std::vector<HostCounters>; return *v; }
struct HostCountersSlot {
    HostCounters h;
    ~HostCountersSlot() {
        if (!h.buf) return;
        std::lock_guard<std::mutex> lk(hc_mu());
        hc_pool().push_back(h);
    }
};
HostCountersSlot& host_counters_slot() {
    thread_local HostCountersSlot slot;
    return slot;
}
HostCounters& host_counters() {
    HostCountersSlot& slot = host_counters_slot();
    if (!slot.h.buf) {
        {
            std::lock_guard<std::mutex> lk(hc_mu());
            auto& pool = hc_pool();
            if (!pool.empty()) {
                slot.h = pool.back();
                pool.pop_back();
            }
        }
        if (!slot.h.buf) {
            // coherent (fine-grained): the device's system-scope stores reach host memory without a cache flush
            if (hipHostMalloc((void**)&slot.h.buf, 64 * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent) !=
                hipSuccess) {
                slot.h.buf = nullptr;
                (void)hipHostMalloc((void**)&slot.h.buf, 64 * sizeof(uint32_t), hipHostMallocDefault);
                slot.h.dev = nullptr;
            }
            else if (hipHostGetDevicePointer((void**)&slot.h.dev, slot.h.buf, 0) != hipSuccess)
                slot.h.dev = nullptr;
            (void)hipEventCreateWithFlags(&slot.h.ev, hipEventDisableTiming);
        }
    }
    return slot.h;
}

// Spin on the sequence word the long-list sort launch writes after the counters (no event: an event record is a
// barrier packet, ~6 us of idle GPU per view).  A fault or a stall ends the spin after 2 s: the stream's error, if any,
// is reported, else the word is re-read once the stream has drained.
// host time spent waiting for the forward's counter read-back, process-wide (dg_host_wait_ns)
std::atomic<uint64_t> g_host_wait_ns{0};

int wait_seq(HostCounters& h, hipStream_t s) {
    volatile uint32_t* w = h.buf + 16;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t it = 0;; it++) {
        if (__atomic_load_n(const_cast<uint32_t*>(w), __ATOMIC_ACQUIRE) == h.seq) return 0;
#if defined(__x86_64__) || defined(__i386__)
        __builtin_ia32_pause();
#else
        if ((it & 63u) == 63u) std::this_thread::yield();
#endif
        if ((it & 4095u) == 4095u && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
    }
    HIP_OK(hipStreamSynchronize(s));
    if (__atomic_load_n(const_cast<uint32_t*>(w), __ATOMIC_ACQUIRE) == h.seq) return 0;
    return fail("forward: the counter read-back never arrived%s%d");
}

// Phase-1 binning capacity, in tile-rect area units (the depth cut bounds the precise instances by the rect areas):
// prefix_per_tile x tiles when > 0, adaptive when 0, everything when < 0.  448 rect units are ~256 precise
// instances per tile on the bench scene.
constexpr int DEFAULT_PREFIX_PER_TILE = 448;
constexpr int MAX_PREFIX_PER_TILE = 8192;
// capacity of any per-instance array: the total rect area bounds every phase's instance count
inline int64_t inst_cap(uint64_t rect) { return (int64_t)(rect < 0xffffff00ull ? (rect ? rect : 1) : 0xffffff00ull); }
bool prefix_enabled(const dg_raster_args* a) { return a->prefix_per_tile >= 0; }
int64_t clamp_cap(int64_t per, int T) {
    const int64_t c = per * (int64_t)T;
    return c < 1 ? 1 : (c > 0xffffff00ll ? 0xffffff00ll : c);
}

// Adaptive phase-1 capacity (prefix_per_tile == 0).  Phase 2 costs 100-400 us whenever it runs, almost independently
// of how many tiles need it (a walk over every Gaussian past the threshold, and the block sort of the few, very long,
// phase-2 lists), so a scene whose views keep leaving tiles unfinished wants a deeper prefix.  Per device and image
// size on this thread: the phase-2 launch leaves its unfinished-tile count in a device probe (k_sat_rows), the next
// forward's k_depth_cut moves it into counters[CNT_PREV_UNF] (cleared after reading), the host sees it in the
// counter copy it makes anyway, and the capacity grows x1.5 (up to MAX_PREFIX_PER_TILE) when it is nonzero -- no
// extra copy, event or wait.  Grow-only: a capacity that was once needed stays, and a too-deep prefix costs only
// proportionally more phase-1 work.  The capacity a view used travels to its backward as the num_instances token, so
// later growth never desynchronises a forward/backward pair.
// The capacity is one state per (device, image size) for the whole process (not per thread), so every thread and
// stream rendering that size shares the growth.  The device probe and the phase-1 count it is judged against are per
// (device, size, stream): a probe is written by one stream's phase 2 and read by that stream's next depth cut, so
// concurrent renders on different streams never read each other's probe (stream order is what makes the pair valid).
struct AdaptiveCap {
    int per_tile = DEFAULT_PREFIX_PER_TILE;
};
struct CapProbe {
    AdaptiveCap* shared = nullptr;
    uint32_t* probe = nullptr;  // device: [0] unfinished tiles, [1] phase-2 instances of the last phase-2 launch
    uint32_t last_e1 = 0;       // phase-1 instances of the last forward at this size on this stream
};
std::mutex g_cap_mu;
// keyed also by the caller's capacity context (dg_raster_args::capacity_ctx; 0: the process-wide default)
using CapKey = std::tuple<int, int, int, int>;
std::map<CapKey, AdaptiveCap>& cap_states() { static auto* m = new std::map<CapKey, AdaptiveCap>; return *m; }
std::map<std::tuple<int, int, int, int, hipStream_t>, CapProbe>& cap_probes() {
    static auto* m = new std::map<std::tuple<int, int, int, int, hipStream_t>, CapProbe>;  // node-based: never move
    return *m;
}
// Released contexts (dg_release_capacity_context): their map nodes are extracted -- so no new render finds them --
// but kept alive until no library call is in flight, since a forward may still hold a CapProbe* of the context.
std::vector<std::map<std::tuple<int, int, int, int, hipStream_t>, CapProbe>::node_type>& cap_probe_graveyard() {
    static auto* v = new std::vector<std::map<std::tuple<int, int, int, int, hipStream_t>, CapProbe>::node_type>;
    return *v;
}
std::vector<std::map<CapKey, AdaptiveCap>::node_type>& cap_state_graveyard() {
    static auto* v = new std::vector<std::map<CapKey, AdaptiveCap>::node_type>;
    return *v;
}

// Library calls in flight, and the shutdown flag (dg_shutdown): a call registers itself before it checks the flag,
// and dg_shutdown sets the flag before it waits for the count to drain, so no call that passed the check can meet
// freed state (the autograd device thread or a ring thread may still be inside the library at exit).
std::atomic<bool> g_shutting_down{false};
std::atomic<int> g_calls_in_flight{0};
struct ApiGuard {
    bool ok;
    ApiGuard() {
        g_calls_in_flight.fetch_add(1, std::memory_order_acq_rel);
        ok = !g_shutting_down.load(std::memory_order_acquire);
    }
    ~ApiGuard() { g_calls_in_flight.fetch_sub(1, std::memory_order_acq_rel); }
    ApiGuard(const ApiGuard&) = delete;
    ApiGuard& operator=(const ApiGuard&) = delete;
};
#define API_GUARD()                                              \
    ApiGuard api_guard_;                                         \
    if (!api_guard_.ok) return fail("the library is shutting down%s%d")

// free the released contexts' probes once this call is the only one in flight (g_cap_mu held)
void drain_cap_graveyard_locked() {
    if (g_calls_in_flight.load(std::memory_order_acquire) > 1) return;
    for (auto& nh : cap_probe_graveyard())
        if (!nh.empty() && nh.mapped().probe) (void)hipFree(nh.mapped().probe);
    cap_probe_graveyard().clear();
    cap_state_graveyard().clear();
}

CapProbe* adaptive_cap(const dg_raster_args* a, hipStream_t s) {
    if (a->prefix_per_tile != 0) return nullptr;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(g_cap_mu);
    CapProbe& c = cap_probes()[std::make_tuple(dev, a->W, a->H, a->capacity_ctx, s)];
    if (!c.probe) {
        c.shared = &cap_states()[std::make_tuple(dev, a->W, a->H, a->capacity_ctx)];
        if (hipMalloc((void**)&c.probe, 2 * sizeof(uint32_t)) != hipSuccess) { c.probe = nullptr; return nullptr; }
        (void)hipMemset(c.probe, 0, 2 * sizeof(uint32_t));
    }
    return &c;
}
int64_t phase1_cap(const dg_raster_args* a, int T, CapProbe* ac) {
    if (a->prefix_per_tile > 0) return clamp_cap(a->prefix_per_tile, T);
    if (!ac) return clamp_cap(DEFAULT_PREFIX_PER_TILE, T);
    std::lock_guard<std::mutex> lk(g_cap_mu);
    return clamp_cap(ac->shared->per_tile, T);
}
// Grow only when the last phase 2 did real work: more than an eighth of phase 1's instances.  Tiles that never
// saturate (sparse regions, the scene's edge seen from a turned camera) stay unfinished at any prefix short of the
// whole list, and phase 2 serves them with a few instances each; growing for them would bin everything
// (measured on the 8-view yaw batch at 1e6: 448 -> 3402 per tile, 1190 -> 843 views/s).
void adapt(CapProbe* ac, uint32_t prev_unfinished, uint32_t prev_k2, uint32_t e1) {
    if (!ac) return;
    std::lock_guard<std::mutex> lk(g_cap_mu);
    const uint32_t prev_e1 = ac->last_e1;
    ac->last_e1 = e1;
    if (prev_unfinished == 0u || (uint64_t)prev_k2 * 8u <= (uint64_t)prev_e1) return;
    int& pt = ac->shared->per_tile;
    if (pt < MAX_PREFIX_PER_TILE) pt = pt * 3 / 2 < MAX_PREFIX_PER_TILE ? pt * 3 / 2 : MAX_PREFIX_PER_TILE;
}

struct BwdScratch {
    float* rec;
    uint2* live_list;                // contributing (slot, Gaussian) per record-sum chunk (k_gauss_sum -> k_gauss_live)
    uint32_t* live_cnt;
    uint32_t* invd_flag;
    size_t bytes;
};
BwdScratch carve_bwd(void* base, int64_t K, int P, int T) {
    Carver c(base);
    BwdScratch s;
    const size_t n = (size_t)(K > 0 ? K : 1);
    s.rec = c.take<float>((size_t)gs::REC_STRIDE * n);
    const size_t chunks = (n + gs::SUM_CHUNK - 1) / gs::SUM_CHUNK;  // every slot < K
    s.live_list = c.take<uint2>(chunks * gs::SUM_CHUNK);
    s.live_cnt = c.take<uint32_t>(chunks);
    s.invd_flag = c.take<uint32_t>(4);
    (void)T;
    s.bytes = c.off;
    return s;
}

void fill_pre(gs::PreArgs& p, const dg_raster_args* a) {
    memset(&p, 0, sizeof(p));
    p.P = a->P; p.D = a->D; p.M = a->M; p.W = a->W; p.H = a->H;
    p.tiles_x = tiles_x_of(a->W); p.tiles_y = tiles_y_of(a->H);
    p.antialiasing = a->antialiasing; p.prefiltered = a->prefiltered;
    p.tanfovx = a->tanfovx; p.tanfovy = a->tanfovy;
    p.focal_y = a->H / (2.0f * a->tanfovy);
    p.focal_x = a->W / (2.0f * a->tanfovx);
    p.scale_mod = a->scale_modifier;
    p.means3D = a->means3D; p.scales = a->scales; p.rotations = a->rotations; p.opacities = a->opacities;
    p.dc = a->dc; p.sh = a->sh; p.colors = a->colors; p.cov3D_precomp = a->cov3D_precomp;
    p.view = a->viewmatrix; p.proj = a->projmatrix; p.campos = a->campos;
    if (p.sh == nullptr || p.M == 0) { p.sh = nullptr; p.D = 0; }
}

int check_args(const dg_raster_args* a) {
    if (!a) return fail("null args%s%d");
    if (a->P < 0 || a->W <= 0 || a->H <= 0) return fail("bad sizes P/W/H%s (P=%d)", "", a->P);
    if (a->P > 0 && (!a->means3D || !a->opacities || !a->viewmatrix || !a->projmatrix || !a->bg))
        return fail("missing required tensor%s%d");
    if (a->P > 0 && !a->colors && (!a->dc || !a->campos))
        return fail("SH path needs dc and campos (or provide colors_precomp)%s%d");
    if (a->P > 0 && !a->cov3D_precomp && (!a->scales || !a->rotations))
        return fail("need scales+rotations or cov3D_precomp%s%d");
    return 0;
}

}  // namespace

extern "C" {

const char* dg_last_error(void) { return g_err.c_str(); }

void dg_profile_enable(int on) { g_prof = on != 0; }

int dg_profile_collect(char* buf, int buflen) {
    // sums per name over everything recorded since the last collect; "name=ms;name=ms;..." (synchronises)
    std::map<std::string, std::pair<double, int>> acc;
    for (auto& r : g_prof_recs) {
        HIP_OK(hipEventSynchronize(r.b));
        float ms = 0.f;
        HIP_OK(hipEventElapsedTime(&ms, r.a, r.b));
        auto& e = acc[r.name];
        e.first += ms;
        e.second += 1;
        g_ev_pool.push_back(r.a);
        g_ev_pool.push_back(r.b);
    }
    g_prof_recs.clear();
    std::string out;
    char tmp[128];
    for (auto& kv : acc) {
        snprintf(tmp, sizeof(tmp), "%s=%.6f/%d;", kv.first.c_str(), kv.second.first, kv.second.second);
        out += tmp;
    }
    if (buf && buflen > 0) {
        strncpy(buf, out.c_str(), (size_t)buflen - 1);
        buf[buflen - 1] = 0;
    }
    return (int)out.size();
}

int dg_sort_pairs_u32(uint32_t* keys, uint32_t* vals, uint32_t n, int begin_bit, int end_bit, dg_alloc_fn alloc,
                      void* user, dg_stream_t stream) {
    if (n == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    Carver c(nullptr);
    c.take<uint32_t>(n); c.take<uint32_t>(n);
    c.take<char>(gs::radix_sort_temp_bytes(n));
    void* base = alloc(user, DG_BUF_TEMP, c.off);
    if (!base) return fail("sort scratch allocation failed%s%d");
    Carver d(base);
    uint32_t* k1 = d.take<uint32_t>(n);
    uint32_t* v1 = d.take<uint32_t>(n);
    void* tmp = d.take<char>(gs::radix_sort_temp_bytes(n));
    const int which = gs::radix_sort_pairs(keys, vals, k1, v1, vals, n, begin_bit, end_bit, tmp, s);
    if (which) {
        HIP_OK(hipMemcpyAsync(keys, k1, 4 * (size_t)n, hipMemcpyDeviceToDevice, s));
        HIP_OK(hipMemcpyAsync(vals, v1, 4 * (size_t)n, hipMemcpyDeviceToDevice, s));
    }
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_exclusive_scan_u32(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* total, dg_alloc_fn alloc,
                          void* user, dg_stream_t stream) {
    void* tmp = alloc(user, DG_BUF_TEMP, gs::scan_temp_bytes(n));
    if (!tmp) return fail("scan scratch allocation failed%s%d");
    gs::exclusive_scan(in, n, out, total, tmp, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}
int dg_version(void) { return 1; }

uint64_t dg_host_wait_ns(void) { return g_host_wait_ns.load(std::memory_order_relaxed); }

// reset / query the adaptive capacity at (device, W, H): ctx < 0 resets every context (state and probes alike) and
// reports context 0; ctx >= 0 only that context
static int adaptive_capacity_impl(int ctx, int W, int H, int reset, int* per_tile_out) {
    int dev = 0;
    HIP_OK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_cap_mu);
    if (reset) {
        for (auto& kv : cap_states())
            if (std::get<0>(kv.first) == dev && std::get<1>(kv.first) == W && std::get<2>(kv.first) == H &&
                (ctx < 0 || std::get<3>(kv.first) == ctx))
                kv.second.per_tile = DEFAULT_PREFIX_PER_TILE;
        for (auto& kv : cap_probes()) {
            if (std::get<0>(kv.first) != dev || std::get<1>(kv.first) != W || std::get<2>(kv.first) != H) continue;
            if (ctx >= 0 && std::get<3>(kv.first) != ctx) continue;
            kv.second.last_e1 = 0;
            if (kv.second.probe) HIP_OK(hipMemset(kv.second.probe, 0, 2 * sizeof(uint32_t)));
        }
    }
    if (per_tile_out) *per_tile_out = cap_states()[std::make_tuple(dev, W, H, ctx < 0 ? 0 : ctx)].per_tile;
    return 0;
}

int dg_adaptive_capacity(int W, int H, int reset, int* per_tile_out) {
    API_GUARD();
    return adaptive_capacity_impl(-1, W, H, reset, per_tile_out);
}

int dg_adaptive_capacity_ctx(int ctx, int W, int H, int reset, int* per_tile_out) {
    API_GUARD();
    if (ctx < 0) return fail("adaptive_capacity_ctx: negative context%s%d");
    return adaptive_capacity_impl(ctx, W, H, reset, per_tile_out);
}

int dg_release_capacity_context(int ctx) {
    API_GUARD();
    if (ctx <= 0) return 0;   // 0 is the process-wide default, never released
    std::lock_guard<std::mutex> lk(g_cap_mu);
    for (auto it = cap_probes().begin(); it != cap_probes().end();) {
        auto nx = std::next(it);
        if (std::get<3>(it->first) == ctx) cap_probe_graveyard().push_back(cap_probes().extract(it));
        it = nx;
    }
    for (auto it = cap_states().begin(); it != cap_states().end();) {
        auto nx = std::next(it);
        if (std::get<3>(it->first) == ctx) cap_state_graveyard().push_back(cap_states().extract(it));
        it = nx;
    }
    drain_cap_graveyard_locked();
    return 0;
}

int dg_capacity_contexts(int* n_out) {
    API_GUARD();
    std::lock_guard<std::mutex> lk(g_cap_mu);
    std::vector<int> seen;
    for (auto& kv : cap_probes()) {
        const int c = std::get<3>(kv.first);
        if (std::find(seen.begin(), seen.end(), c) == seen.end()) seen.push_back(c);
    }
    if (n_out) *n_out = (int)seen.size();
    return 0;
}

uint64_t dg_geom_bytes(int P) { return carve_geom(nullptr, P).bytes; }
uint64_t dg_image_bytes(int W, int H) { return carve_image(nullptr, W, H).bytes; }
uint64_t dg_binning_bytes(int64_t K, int W, int H) { (void)W; (void)H; return carve_binning(nullptr, K).bytes; }

uint64_t dg_backward_scratch_bytes(const dg_raster_args* a, int64_t num_rendered) {
    if (!a || a->P <= 0 || num_rendered < 0) return 0;
    const int T = tiles_x_of(a->W) * tiles_y_of(a->H);
    return carve_bwd(nullptr, inst_cap((uint64_t)num_rendered), a->P, T).bytes;
}

void* dg_fixed_alloc(void* user, int which, uint64_t nbytes) {
    (void)which;
    const dg_fixed_buffer* f = static_cast<const dg_fixed_buffer*>(user);
    if (!f || !f->ptr || nbytes > f->bytes) {
        fail("fixed buffer too small for the request (%s%d MiB held)", "", f ? (int)(f->bytes >> 20) : 0);
        return nullptr;
    }
    return f->ptr;
}

}  // extern "C"

namespace {
// Rasterizer::forward (rasterizer_impl.cu:334-498); gcount (optional): count mode, contributing pixels per Gaussian
// The native step's activation fold: the preprocess reads the raw parameters and writes the activated ones to
// a->opacities / scales / rotations (PreArgs::raw_*), plus the regulariser's per-block partial sums.
struct ActFold {
    const float *raw_o, *raw_s, *raw_q;
    float* part_sc;
    uint64_t* zero_stamp;         // *zero_stamp = stamp when some activated scaling is 0 (the regulariser's backward)
    uint64_t stamp;
    hipEvent_t wait_before_emit;  // optional: the previous step's overlapped SH update (the emission reads the SH)
    bool waited;                  // out: the wait was enqueued (a forward that binned nothing leaves it to the caller)
};

int forward_impl(const dg_raster_args* a, float* out_color, float* out_invdepth, int* radii, dg_alloc_fn alloc,
                 void* user, void** geom_out, void** binning_out, void** image_out, void** binning2_out,
                 int64_t* num_rendered, int64_t* num_instances, dg_stream_t stream_, uint32_t* gcount,
                 ActFold* fold = nullptr) {
    if (check_args(a)) return 1;
    hipStream_t s = (hipStream_t)stream_;
    const int P = a->P, W = a->W, H = a->H;
    const int tx = tiles_x_of(W), ty = tiles_y_of(H), T = tx * ty;
    *num_rendered = 0;
    *num_instances = 0;
    *binning_out = nullptr;
    *binning2_out = nullptr;

    CapProbe* const ac = adaptive_cap(a, s);
    const size_t gbytes = carve_geom(nullptr, P).bytes;
    void* gbase = alloc(user, DG_BUF_GEOM, gbytes);
    if (!gbase) return fail("geometry allocation failed%s%d");
    Geom g = carve_geom(gbase, P);
    const size_t ibytes = carve_image(nullptr, W, H).bytes;
    void* ibase = alloc(user, DG_BUF_IMAGE, ibytes);
    if (!ibase) return fail("image allocation failed%s%d");
    Image im = carve_image(ibase, W, H);
    *geom_out = gbase;
    *image_out = ibase;

    // no memset of the counters: k_depth_cut writes every slot (the preprocess's sums and error bits go through
    // its per-block parts)
    gs::PreArgs pre;
    fill_pre(pre, a);
    if (fold) {
        pre.raw_o = fold->raw_o; pre.raw_s = fold->raw_s; pre.raw_q = fold->raw_q; pre.part_sc = fold->part_sc;
        pre.zero_stamp = fold->zero_stamp; pre.stamp = fold->stamp;
    }
    pre.radii = radii; pre.sp = g.sp; pre.depthkey = g.dkey; pre.cnt = g.cnt; pre.rcnt = g.rcnt;
    pre.hist = g.hist;
    pre.unf_rows = UNF_ROWS ? reinterpret_cast<unsigned long long*>(im.sat) : nullptr;  // (the SAT block is larger)
    pre.unf_words = UNF_ROWS ? (ty + 1) * unf_rw_of(tx) + (ty + 63) / 64 : 0;  // rows, column OR, row summary
    // per-block rect sums land in the wave-total array (ceil(P/64) u32 >= ceil(P/256) u64), free until the binning
    pre.rect_part = reinterpret_cast<unsigned long long*>(g.wtot); pre.err = g.counters + gs::CNT_ERR;
    const uint32_t nparts = gs::preprocess_blocks(P);
    { PROF("preprocess"); gs::launch_preprocess(pre, s); }
    DBG_SYNC(a->debug, s);

    // ---- depth-threshold prefix: histogram of tile-rect areas over depth bins -> threshold (no depth sort)
    int64_t C1;
    if (P == 0) HIP_OK(hipMemsetAsync(g.hist, 0, gs::DH_BINS * sizeof(uint32_t), s));  // no preprocess to zero it
    {
        PROF("prefix_cut");
        if (prefix_enabled(a)) {
            C1 = phase1_cap(a, T, ac);
            gs::launch_depth_hist_cut(P, g.dkey, g.cnt, g.hist, (uint32_t)C1, g.counters, im.tile_cnt, im.tile_cnt2,
                                      (uint32_t)T, pre.rect_part, nparts, ac ? ac->probe : nullptr, s);
        } else {  // everything in one phase: the capacity is the total rect area itself (one early sync)
            gs::launch_depth_hist_cut(P, g.dkey, g.cnt, g.hist, 0xffffffffu, g.counters, im.tile_cnt, im.tile_cnt2,
                                      (uint32_t)T, pre.rect_part, nparts, nullptr, s);
            uint32_t k = 0;
            HIP_OK(hipMemcpyAsync(&k, g.counters + gs::CNT_K, 4, hipMemcpyDeviceToHost, s));
            HIP_OK(hipStreamSynchronize(s));
            C1 = k;
        }
    }
    DBG_SYNC(a->debug, s);

    const size_t bbytes = carve_binning(nullptr, C1).bytes;
    void* bbase = alloc(user, DG_BUF_BINNING, bbytes);
    if (!bbase) return fail("binning allocation failed%s%d");
    *binning_out = bbase;
    Binning b = carve_binning(bbase, C1);
    // the native step's overlapped SH update (fold->wait_before_emit): the phase-1 emission runs without the colours,
    // and the colour pass waits for the update after the long-list sort (below)
    hipEvent_t sh_wait = fold ? fold->wait_before_emit : nullptr;
    gs::BinArgs ba1;
    const bool colors_later = sh_wait && C1 > 0 && P > 0;
    if (C1 > 0 && P > 0) {
        ba1 = bin_args(a, g, im, T, (uint32_t)C1, b, im.tile_cnt, im.ranges);
        ba1.colors_later = colors_later ? 1 : 0;
        { PROF("emit"); gs::launch_bin(1, ba1, g.counters + gs::CNT_E1, g.scan_tmp, s); }
        DBG_SYNC(a->debug, s);
    }
    // the host's only wait is on this early copy (num_rendered, E1, error flag, cut), and it happens after all of
    // phase 1 is queued, so the GPU never idles on it
    HostCounters& hcs = host_counters();
    const gs::DSortArgs ds1 = dsort_args(b, C1, T, im.ranges, nullptr, nullptr, im.long_tiles,
                                         g.counters + gs::CNT_LONG);
    // the phase-1 render lands the counters in the pinned buffer itself (no copy launch, no event: ~6-10 us of idle
    // GPU per view); without a device-addressable buffer, a copy and an event
#ifdef DG_HC_MEMCPY  // A/B switch: the copy launch
    const bool kcopy = false;
#else
    const bool kcopy = hcs.dev != nullptr && T > 0;
#endif
    if (!kcopy) {
        HIP_OK(hipMemcpyAsync(hcs.buf, g.counters, 16 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIP_OK(hipEventRecord(hcs.ev, s));
    }
    const bool fuse = FUSED_SORT && C1 > 0 && P > 0;
    if (C1 > 0 && P > 0) {
        // the lists longer than a wave's capacity here; the render sorts the others tile by tile (fused)
        { PROF("tile_bin"); if (fuse) gs::tile_depth_sort_long_only(ds1, s); else gs::tile_depth_sort(ds1, s); }
        DBG_SYNC(a->debug, s);
    } else {
        HIP_OK(hipMemsetAsync(im.ranges, 0, sizeof(uint2) * (size_t)T, s));
    }
    if (colors_later) {
        HIP_OK(hipStreamWaitEvent(s, sh_wait, 0));
        fold->waited = true;
        sh_wait = nullptr;
        gs::launch_binned_colors(ba1, s);
    }

    gs::RenderArgs r;
    memset(&r, 0, sizeof(r));
    r.W = W; r.H = H; r.tiles_x = tx; r.num_tiles = T;
    r.K = (uint32_t)(C1 > 0 ? C1 : 1); r.P = (uint32_t)(P > 0 ? P : 1);
    r.ranges = im.ranges; r.s_e = b.se; r.eg = b.eg; r.sp = g.sp; r.rgbi = g.rgbi; r.bg = a->bg;
    r.out_color = out_color; r.out_invd = out_invdepth; r.final_T = im.final_T; r.img_color = im.img_color;
    r.img_invd = im.img_invd; r.n_contrib = im.n_contrib; r.max_contrib = im.max_contrib;
    r.phase = 1; r.counters = g.counters; r.unfinished = im.unfinished; r.resume = im.resume;
    r.unf_list = im.unf_list;
    r.ranges2_zero = im.ranges2;
    r.unf_rows = pre.unf_rows; r.unf_rw = unf_rw_of(tx);
    r.gcount = gcount;
    r.fuse_sort = fuse ? 1 : 0;
    r.ds = ds1;
    if (kcopy) { r.hc_src = g.counters; r.hc_dst = hcs.dev; r.hc_seq = ++hcs.seq; }
    if (gcount && P > 0) HIP_OK(hipMemsetAsync(gcount, 0, sizeof(uint32_t) * (size_t)P, s));
    { PROF("render_fwd"); gs::launch_render_fwd(r, s); }
    DBG_SYNC(a->debug, s);

    {
        const auto w0 = std::chrono::steady_clock::now();
        if (kcopy) {
            if (wait_seq(hcs, s)) return 1;
        } else {
            HIP_OK(hipEventSynchronize(hcs.ev));
        }
        g_host_wait_ns.fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                     std::chrono::steady_clock::now() - w0).count(), std::memory_order_relaxed);
    }
    const uint32_t* hc = hcs.buf;
    adapt(ac, hc[gs::CNT_PREV_UNF], hc[gs::CNT_PREV_K2], hc[gs::CNT_E1]);
    if (hc[gs::CNT_ERR]) return fail("a Gaussian was filtered although prefiltered is set%s%d");
    const uint64_t rect = (uint64_t)hc[gs::CNT_RECT_LO] | ((uint64_t)hc[gs::CNT_RECT_LO + 1] << 32);
    *num_rendered = (int64_t)rect;
    // the num_buckets slot: the phase-1 capacity this view was binned with (the backward carves the phase-1 block
    // at it; with the adaptive policy it can change between views).  Phase 2 and the backward's per-instance state
    // are sized by num_rendered, which bounds phase 1 + phase 2.
    *num_instances = C1;
    if (!hc[gs::CNT_CUT]) {
        HIP_OK(hipGetLastError());
        return 0;
    }

    // ---- phase 2: the Gaussians past the threshold, only for tiles phase 1 left unfinished.  Every kernel is gated
    // on the device-side unfinished count, so nothing waits for phase 1 and the common case costs a few empty launches.
    const int64_t K = inst_cap(rect);
    const size_t b2bytes = carve_binning(nullptr, K).bytes;
    void* b2base = alloc(user, DG_BUF_BINNING2, b2bytes);
    if (!b2base) return fail("phase-2 binning allocation failed%s%d");
    *binning2_out = b2base;
    Binning b2 = carve_binning(b2base, K);
    const uint32_t* gate = g.counters + gs::CNT_UNFINISHED;
    {
        PROF("phase2");
        if (!UNF_ROWS) gs::launch_unfinished_sat(g.counters, im.unfinished, tx, ty, im.sat, s, ac ? ac->probe : nullptr);
        gs::BinArgs ba = bin_args(a, g, im, T, (uint32_t)K, b2, im.tile_cnt2, im.ranges2);
        ba.unf_rows = UNF_ROWS ? reinterpret_cast<const unsigned long long*>(im.sat) : nullptr;
        ba.unf_rw = unf_rw_of(tx); ba.unf_th = ty;
        ba.probe = UNF_ROWS && ac ? ac->probe : nullptr;
        const bool multi_order = gs::render_fwd2_orders() && gs::bin_emit_orders();
        if (multi_order) {
            ba.ohist = im.ohist; ba.max_contrib = im.max_contrib; ba.ranges1 = im.ranges;
            ba.unf_list = im.unf_list; ba.unf_sorted = im.unf_sorted;
        }
        gs::launch_bin(2, ba, g.counters + gs::CNT_K2, g.scan_tmp, s, sh_wait);
        if (sh_wait) fold->waited = true;
        sh_wait = nullptr;
        const gs::DSortArgs ds2 = dsort_args(b2, K, T, im.ranges2, im.unfinished, gate, im.long_tiles,
                                             g.counters + gs::CNT_LONG2);
        gs::RenderArgs r2 = r;
#if defined(DG_PHASE2_WAVE_PER_TILE) || defined(DG_PHASE2_STANDALONE_SORT)
        gs::tile_depth_sort(ds2, s);
        r2.fuse_sort = 0;
#else
        r2.fuse_sort = 1;  // k_render_fwd2 sorts its tile's list itself
#endif
        r2.ds = ds2;
        r2.phase = 2;
        r2.K = (uint32_t)K;
        r2.ranges = im.ranges2; r2.ranges1 = im.ranges; r2.s_e = b2.se; r2.eg = b2.eg;
        r2.probe = ac ? ac->probe : nullptr;
        r2.order = im.order;
        r2.ohist = multi_order ? im.ohist : nullptr;
        r2.unf_sorted = multi_order ? im.unf_sorted : nullptr;
        gs::launch_render_fwd(r2, s);
    }
    DBG_SYNC(a->debug, s);
    HIP_OK(hipGetLastError());
    return 0;
}

}  // namespace

extern "C" {

int dg_rasterize_forward(const dg_raster_args* a, float* out_color, float* out_invdepth, int* radii,
                         dg_alloc_fn alloc, void* user, void** geom_out, void** binning_out, void** image_out,
                         void** binning2_out, int64_t* num_rendered, int64_t* num_instances, dg_stream_t stream) {
    API_GUARD();
    return forward_impl(a, out_color, out_invdepth, radii, alloc, user, geom_out, binning_out, image_out,
                        binning2_out, num_rendered, num_instances, stream, nullptr);
}

int dg_rasterize_count(const dg_raster_args* a, float* out_color, int* radii, int32_t* gaussians_count,
                       float* important_score, dg_alloc_fn alloc, void* user, int64_t* num_rendered,
                       dg_stream_t stream) {
    API_GUARD();
    if (check_args(a)) return 1;
    if (a->P > 0 && (!gaussians_count || !important_score)) return fail("count outputs required%s%d");
    hipStream_t s = (hipStream_t)stream;
    const size_t HW = (size_t)a->W * a->H;
    float* invd = nullptr;
    HIP_OK(hipMallocAsync((void**)&invd, (HW ? HW : 1) * sizeof(float), s));
    void *g = nullptr, *b = nullptr, *im = nullptr, *b2 = nullptr;
    int64_t ninst = 0;
    const int rc = forward_impl(a, out_color, invd, radii, alloc, user, &g, &b, &im, &b2, num_rendered, &ninst, stream,
                                reinterpret_cast<uint32_t*>(gaussians_count));
    if (rc == 0 && a->P > 0)
        gs::launch_count_score(a->P, radii, carve_geom(g, a->P).sp, reinterpret_cast<const uint32_t*>(gaussians_count),
                               important_score, s);
    HIP_OK(hipFreeAsync(invd, s));
    if (rc) return rc;
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_rasterize_backward(const dg_raster_args* a, const int* radii, const void* geom, const void* binning,
                          const void* image, const void* binning2, int64_t num_rendered, int64_t K,
                          const float* dL_dout_color, const float* dL_dout_invdepth, float* dmeans2D, float* dcolors,
                          float* dopacity, float* dmeans3D, float* dcov3D, float* ddc, float* dsh, float* dscales,
                          float* drot, float* depth, dg_alloc_fn alloc, void* user, dg_stream_t stream_) {
    API_GUARD();
    if (check_args(a)) return 1;
    hipStream_t s = (hipStream_t)stream_;
    const int P = a->P, W = a->W, H = a->H;
    const int tx = tiles_x_of(W), ty = tiles_y_of(H), T = tx * ty;
    if (P == 0) return 0;
    Geom g = carve_geom((void*)geom, P);
    Image im = carve_image((void*)image, W, H);
    // the phase-1 block was carved at C1 = the forward's num_instances token, the phase-2 block at the rect total
    const int64_t Kcap = inst_cap((uint64_t)num_rendered);
    const int64_t C1 = K;
    if (C1 < 0 || C1 > Kcap + (prefix_enabled(a) ? clamp_cap(MAX_PREFIX_PER_TILE, T) : 0))
        return fail("num_instances is not the forward's token%s (%d)", "", (int)C1);
    Binning b = carve_binning((void*)binning, C1);
    const uint32_t* s_e = b.se;
    const uint32_t* s_e2 = nullptr;
    const uint32_t* eg2 = nullptr;
    uint8_t* flag2 = nullptr;
    if (binning2) {
        Binning b2 = carve_binning((void*)binning2, Kcap);
        s_e2 = b2.se;
        eg2 = b2.eg;
        flag2 = b2.flag;
    }

    const size_t sbytes = carve_bwd(nullptr, Kcap, P, T).bytes;
    void* sbase = alloc(user, DG_BUF_BACKWARD, sbytes);
    if (!sbase) return fail("backward scratch allocation failed%s%d");
    BwdScratch sc = carve_bwd(sbase, Kcap, P, T);
    if (a->M > 0 && !dsh) return fail("dsh output required when M > 0%s%d");
    // the nine gradient outputs back to back (the Python side allocates them as views of one buffer): the replay
    // zero-fills them while it is VALU-bound; otherwise the aux blocks of k_gauss_sum do
    size_t zero_count = 0;
    {
        const size_t Pz = (size_t)P, Mz = (size_t)(a->M > 0 ? a->M : 0);
        float* const ptrs[9] = {dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, ddc, dsh, dscales, drot};
        const size_t counts[9] = {3 * Pz, 3 * Pz, Pz, 3 * Pz, 6 * Pz, 3 * Pz, 3 * Mz * Pz, 3 * Pz, 4 * Pz};
        bool adjacent = (reinterpret_cast<uintptr_t>(dmeans2D) & 15u) == 0u;
        size_t total = counts[0];
        for (int i = 1; i < 9; i++) {
            adjacent = adjacent && (counts[i] == 0 || ptrs[i] == dmeans2D + total);
            total += counts[i];
        }
        if (adjacent) zero_count = total;
#ifdef DG_NO_ZERO_FILL  // timing experiment only (tools/gpu_r5be.sh): no zero fill anywhere, wrong non-contributing rows
        zero_count = 0;
#endif
    }
    {
        gs::RenderBwdArgs r;
        r.zero_base = zero_count ? dmeans2D : nullptr; r.zero_count = zero_count;
        r.W = W; r.H = H; r.tiles_x = tx; r.num_tiles = T;
        r.K = (uint32_t)Kcap; r.K1 = (uint32_t)C1; r.P = (uint32_t)P;
        r.ranges = im.ranges; r.max_contrib = im.max_contrib; r.s_e = s_e; r.eg = b.eg;
        r.ranges2 = binning2 ? im.ranges2 : nullptr; r.s_e2 = s_e2; r.eg2 = eg2; r.counters = g.counters;
        r.unfinished = im.unfinished;
        r.sp = g.sp; r.rgbi = g.rgbi; r.bg = a->bg;
        r.final_T = im.final_T; r.img_color = im.img_color; r.img_invd = im.img_invd; r.n_contrib = im.n_contrib;
        r.dL_dpix = dL_dout_color; r.dL_dinvd = dL_dout_invdepth; r.rec = sc.rec; r.flag = b.flag; r.flag2 = flag2;
        r.order = im.order;
        { PROF("render_bwd"); gs::launch_render_bwd(r, g.counters, s, binning2 != nullptr && gs::render_fwd2_orders()); }
        DBG_SYNC(a->debug, s);
    }
    gs::GaussBwdArgs q;
    memset(&q, 0, sizeof(q));
    q.P = P; q.D = a->D; q.M = a->M; q.W = W; q.H = H; q.antialiasing = a->antialiasing;
    q.K = (uint32_t)Kcap;
    q.tanfovx = a->tanfovx; q.tanfovy = a->tanfovy;
    q.focal_y = H / (2.0f * a->tanfovy);
    q.focal_x = W / (2.0f * a->tanfovx);
    q.scale_mod = a->scale_modifier;
    q.means3D = a->means3D; q.scales = a->scales; q.rotations = a->rotations; q.opacities = a->opacities;
    q.dc = a->dc; q.sh = (a->M > 0) ? a->sh : nullptr; q.cov3D_precomp = a->cov3D_precomp;
    q.view = a->viewmatrix; q.proj = a->projmatrix; q.campos = a->campos;
    q.radii = radii; q.dkey = g.dkey; q.sp = g.sp; q.rec = sc.rec; q.flag = b.flag; q.flag2 = flag2;
    q.eg = b.eg; q.eg2 = eg2; q.counters = g.counters; q.K1 = (uint32_t)C1;
    q.dmeans2D = dmeans2D; q.dcolors = dcolors; q.dopacity = dopacity; q.dmeans3D = dmeans3D; q.dcov3D = dcov3D;
    q.ddc = ddc; q.dsh = dsh; q.dscales = dscales; q.drot = drot; q.depth = depth;
    q.live_list = sc.live_list; q.live_cnt = sc.live_cnt;
#ifdef DG_NO_ZERO_FILL
    q.outputs_zeroed = true;
#else
    q.outputs_zeroed = zero_count != 0;
#endif
    { PROF("gauss_bwd"); gs::launch_gauss_bwd(q, s); }
    DBG_SYNC(a->debug, s);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix, uint8_t* present,
                    dg_stream_t stream) {
    (void)projmatrix;
    gs::launch_mark_visible(P, means3D, viewmatrix, (bool*)present, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

size_t dg_conv3x3_wgrad_scratch_bytes(int Cin, int Cout, int H, int W) {
    if (Cin < 1 || Cout < 1 || H < 1 || W < 1) return 0;
    return gs::conv3x3_wgrad_scratch_bytes(Cin, Cout, H, W);
}

int dg_conv3x3_wgrad(int Cin, int Cout, int H, int W, const float* x, const float* dy, const float* gate, int flags,
                     float* dw, float* db, void* scratch, size_t scratch_bytes, dg_stream_t stream) {
    if ((flags & ~DG_CONV_SHUFFLE) || ((flags & DG_CONV_SHUFFLE) && ((H | W) & 1)))
        return fail("conv3x3_wgrad: bad flags%s%d");
    if (H < 1 || W < 1 || !x || !dy || !dw || !db || !scratch) return fail("conv3x3_wgrad: bad args%s%d");
    if (!gs::conv3x3_wgrad_supported(Cin, Cout)) return fail("conv3x3_wgrad: unsupported channel counts%s%d", "", Cin * Cout);
    if (scratch_bytes < gs::conv3x3_wgrad_scratch_bytes(Cin, Cout, H, W))
        return fail("conv3x3_wgrad: scratch too small%s%d");
    gs::launch_conv3x3_wgrad(Cin, Cout, H, W, x, dy, gate, (flags & DG_CONV_SHUFFLE) != 0, dw, db, (float*)scratch,
                             (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_conv3x3(int Cin, int Cout, int H, int W, const float* x, const float* w, const float* b, float* y, int flags,
               const float* gate, dg_stream_t stream) {
    if (!x || !w || !y || (flags & ~7)) return fail("conv3x3: bad args%s%d");
    if ((flags & DG_CONV_SHUFFLE) && ((H | W) & 1)) return fail("conv3x3: odd size with DG_CONV_SHUFFLE%s%d");
    if (!gs::conv3x3_supported(Cin, Cout, H, W)) return fail("conv3x3: unsupported shape%s%d", "", Cin * Cout);
    const bool sh = (flags & DG_CONV_SHUFFLE) != 0;
    // the adjoint launches Cout -> Cin over the forward's weights
    if (flags & DG_CONV_ADJOINT)
        gs::launch_conv3x3(Cout, Cin, H, W, x, w, nullptr, y, true, false, gate, sh, (hipStream_t)stream);
    else
        gs::launch_conv3x3(Cin, Cout, H, W, x, w, b, y, false, (flags & DG_CONV_RELU) != 0, nullptr, sh,
                           (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

static bool head_shape_ok(int H, int W, int h2, int w2) {
    // the adjoint gather lists at most 12 samples per source index and axis: upsampling by at most 4
    return H > 0 && W > 0 && h2 > 0 && w2 > 0 && H <= 4 * h2 && W <= 4 * w2;
}

static gs::HeadArgs head_args(int H, int W, int h2, int w2, const float* u, const float* w1, const float* b1,
                              const float* w2p, const float* b2) {
    gs::HeadArgs a = {};
    a.H = H; a.W = W; a.h2 = h2; a.w2 = w2;
    a.sh = (float)h2 / (float)H; a.sw = (float)w2 / (float)W;
    a.U = u; a.k1 = w1; a.b1 = b1; a.k2 = w2p; a.b2 = b2;
    return a;
}

int dg_mask_head_forward(int H, int W, int h2, int w2, const float* u, const float* w1, const float* b1,
                         const float* w2p, const float* b2, float* mask, float* hidden, dg_stream_t stream) {
    if (!head_shape_ok(H, W, h2, w2) || !u || !w1 || !b1 || !w2p || !b2 || !mask)
        return fail("mask_head_forward: bad args%s%d");
    gs::HeadArgs a = head_args(H, W, h2, w2, u, w1, b1, w2p, b2);
    a.mask = mask;
    a.hid = hidden;
    gs::launch_mask_head_fwd(a, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

size_t dg_mask_head_scratch_bytes(int H, int W) {
    if (H < 1 || W < 1) return 0;
    const size_t HW = (size_t)H * W;
    return (24 * HW + (size_t)gs::mask_head_tiles(H, W) * gs::mask_head_nparams() +
            gs::rowsum_scratch_floats(gs::mask_head_tiles(H, W), gs::mask_head_nparams())) * sizeof(float);
}

int dg_mask_head_nparams(void) { return gs::mask_head_nparams(); }

int dg_mask_head_backward(int H, int W, int h2, int w2, const float* u, const float* w1, const float* b1,
                          const float* w2p, const float* b2, const float* dmask, const float* hidden, float* du,
                          float* dparams, void* scratch, size_t scratch_bytes, dg_stream_t stream) {
    if (!head_shape_ok(H, W, h2, w2) || !u || !w1 || !b1 || !w2p || !b2 || !dmask || !du || !dparams || !scratch)
        return fail("mask_head_backward: bad args%s%d");
    if (scratch_bytes < dg_mask_head_scratch_bytes(H, W)) return fail("mask_head_backward: scratch too small%s%d");
    gs::HeadArgs a = head_args(H, W, h2, w2, u, w1, b1, w2p, b2);
    const size_t HW = (size_t)H * W;
    float* f = (float*)scratch;
    a.dmask = dmask; a.dh = f; a.dx = f + 8 * HW; a.part = f + 24 * HW; a.du = du;
    a.hid = const_cast<float*>(hidden);
    gs::launch_mask_head_bwd(a, dparams, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_cull_log_threshold(int64_t n, const float* opacity, float* thr, dg_stream_t stream) {
    if (n < 0 || (n > 0 && (!opacity || !thr))) return fail("bad args%s%d");
    gs::launch_cull_log_threshold(n, opacity, thr, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_rasterize_filter(const dg_raster_args* a, int* radii, dg_stream_t stream) {
    if (!a || a->P < 0) return fail("bad args%s%d");
    if (a->P == 0) return 0;
    gs::PreArgs p;
    fill_pre(p, a);
    p.radii = radii;
    uint32_t* err = nullptr;
    HIP_OK(hipMallocAsync((void**)&err, 4, (hipStream_t)stream));
    HIP_OK(hipMemsetAsync(err, 0, 4, (hipStream_t)stream));
    p.err = err;
    gs::launch_filter(p, (hipStream_t)stream);
    uint32_t h = 0;
    HIP_OK(hipMemcpyAsync(&h, err, 4, hipMemcpyDeviceToHost, (hipStream_t)stream));
    HIP_OK(hipFreeAsync(err, (hipStream_t)stream));
    HIP_OK(hipStreamSynchronize((hipStream_t)stream));
    if (h) return fail("a Gaussian was filtered although prefiltered is set%s%d");
    HIP_OK(hipGetLastError());
    return 0;
}

// The native step's overlapped SH update (dg_train_step_args::sh_status): per caller stream, a side stream and the
// event its f_dc / f_rest update records; `pending` until a later step (or dg_train_sync) made the stream wait on it.
}  // extern "C"

namespace {
// blocks of the side launch: few enough that the overlapped forward's kernels find free compute units
uint32_t sh_grid_cap() {
    static const uint32_t v = [] {
        const char* e = getenv("DG_SH_ADAM_BLOCKS");
        return e ? (uint32_t)atoi(e) : 0u;
    }();
    return v;
}
struct ShOverlap {
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, done = nullptr;
    bool pending = false;
};
std::mutex& sh_mu() { static auto* m = new std::mutex; return *m; }
std::map<hipStream_t, ShOverlap>& sh_map() { static auto* m = new std::map<hipStream_t, ShOverlap>; return *m; }
ShOverlap* sh_state(hipStream_t s, bool create) {
    std::lock_guard<std::mutex> lk(sh_mu());
    auto& mp = sh_map();
    auto it = mp.find(s);
    if (it != mp.end()) return &it->second;
    if (!create) return nullptr;
    ShOverlap o;
    // the side stream at the lowest priority: the dispatcher then prefers the overlapped forward's work groups (at
    // equal priority the update's many small groups kept a one-block launch of the forward waiting ~150 us)
    int least = 0, greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (const char* e = getenv("DG_SH_PRIO")) least = atoi(e);
    if (hipStreamCreateWithPriority(&o.side, hipStreamNonBlocking, least) != hipSuccess) return nullptr;
    if (hipEventCreateWithFlags(&o.fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&o.done, hipEventDisableTiming) != hipSuccess)
        return nullptr;
    return &(mp[s] = o);
}
}  // namespace

extern "C" {

static int fill_stats(gs::AdamMultiArgs& m, const dg_densify_stats* st) {
    if (!st) return 0;
    if (!st->radii || !st->dmeans2D || !st->max_radii2D || !st->grad_accum || !st->denom)
        return fail("densification statistics need radii, dmeans2D, max_radii2D, grad_accum and denom%s%d");
    if (st->dmeans2D_stride < 2) return fail("dmeans2D_stride must be >= 2%s%d");
    m.radii = st->radii; m.dmeans2D = st->dmeans2D; m.dm_stride = st->dmeans2D_stride;
    m.max_radii2D = st->max_radii2D; m.grad_accum = st->grad_accum; m.denom = st->denom;
    return 0;
}

int dg_adam_update_groups(const dg_adam_group* groups, int n_groups, const uint8_t* visible, uint32_t N, float b1,
                          float b2, const dg_densify_stats* stats, dg_stream_t stream) {
    return dg_adam_update_groups_prox(groups, nullptr, n_groups, visible, N, b1, b2, stats, stream);
}

int dg_adam_update_groups_prox(const dg_adam_group* groups, const dg_adam_prox* prox, int n_groups,
                               const uint8_t* visible, uint32_t N, float b1, float b2, const dg_densify_stats* stats,
                               dg_stream_t stream) {
    if (n_groups < 0 || n_groups > gs::MAX_ADAM_GROUPS) return fail("n_groups must be 0..8%s (got %d)", "", n_groups);
    if (N && !visible) return fail("visible mask required%s%d");
    gs::AdamMultiArgs m;
    memset(&m, 0, sizeof(m));
    m.visible = visible; m.N = N; m.b1 = b1; m.b2 = b2;
    int n = 0;
    for (int k = 0; k < n_groups; k++) {
        const dg_adam_group& g = groups[k];
        if (g.M == 0) continue;
        if (!g.param || !g.grad || !g.exp_avg || !g.exp_avg_sq) return fail("adam group %s%d has a NULL tensor", "", k);
        if ((uint64_t)N * g.M >= 0xfffff000ull) return fail("adam group %s%d: N * M must be < 2^32", "", k);
        gs::AdamGroup& d = m.g[n++];
        d.param = g.param; d.grad = g.grad; d.m = g.exp_avg; d.v = g.exp_avg_sq; d.lr = g.lr; d.eps = g.eps; d.M = g.M;
        const uintptr_t al = reinterpret_cast<uintptr_t>(g.param) | reinterpret_cast<uintptr_t>(g.grad) |
                             reinterpret_cast<uintptr_t>(g.exp_avg) | reinterpret_cast<uintptr_t>(g.exp_avg_sq);
        uintptr_t alp = 0;
        if (prox && prox[k].u) {
            if (!prox[k].z) return fail("adam group %s%d: prox u without z", "", k);
            d.u = prox[k].u; d.z = prox[k].z; d.coef = prox[k].coef;
            alp = reinterpret_cast<uintptr_t>(prox[k].u) | reinterpret_cast<uintptr_t>(prox[k].z);
        }
        d.vec = ((al | alp) & 15u) == 0u;
    }
    m.n = n;
    if (fill_stats(m, stats)) return 1;
    if (N) gs::launch_adam_multi(m, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_train_step(const dg_train_step_args* a, dg_alloc_fn alloc, void* user, dg_stream_t stream) {
    API_GUARD();
    if (!a || !a->gt || !a->radii || !a->image) return fail("train step: args, gt, radii and image are required%s%d");
    hipStream_t s = (hipStream_t)stream;
    const int P = a->view.P, W = a->view.W, H = a->view.H, M = a->view.M;
    if (P <= 0 || W <= 0 || H <= 0) return fail("train step: empty model or image%s (P=%d)", "", P);
    for (int k = 0; k < 6; k++)
        if (!a->groups[k].param || !a->groups[k].exp_avg || !a->groups[k].exp_avg_sq)
            return fail("train step: group %s%d lacks param or moments", "", k);
    const size_t Pz = (size_t)P, Mz = (size_t)(M > 0 ? M : 0), n_img = 3 * (size_t)W * H, HW = (size_t)W * H;
    if (n_img >= 0xffffff00ull) return fail("train step: image too large%s%d");
    const uint32_t nb_l1 = gs::clamp_l1_blocks((uint32_t)n_img);
    const uint32_t nb_map = gs::block_sum_blocks((uint32_t)n_img), nb_sc = gs::block_sum_blocks((uint32_t)P);
    const uint32_t nw_ssim = gs::ssim_waves(3, H, W);  // the fused SSIM's partials: nw L1, then nw map
    const uint32_t nb_act = gs::preprocess_blocks(P);  // the fused route's regulariser partials (preprocess blocks)
    // fused route: nw L1 partials, nw map partials, nw mask-regulariser partials, then the regulariser's
    const uint32_t n_part = (nb_l1 + nb_map > 3 * nw_ssim ? nb_l1 + nb_map : 3 * nw_ssim) + (nb_sc > nb_act ? nb_sc : nb_act);
    if (a->mask && (!a->dmask || ((reinterpret_cast<uintptr_t>(a->mask) | reinterpret_cast<uintptr_t>(a->dmask)) & 15u)))
        return fail("train step: a mask needs a dmask output, both 16-byte aligned%s%d");
    if (a->mask && getenv("DG_TRAIN_UNFUSED")) return fail("train step: the appearance mask needs the fused route%s%d");
    // ---- the step's scratch (DG_BUF_TRAIN).  The nine rasterizer gradients (back to back: the replay zero-fills them)
    // come first: the overlapped f_dc / f_rest update still reads ddc / dsh while the next step's forward writes this
    // block, so their offsets must not depend on the image size (the arena hands the same block back to a view of
    // another size whenever it fits)
    const size_t n9 = (3 + 3 + 1 + 3 + 6 + 3 + 3 * Mz + 3 + 4) * Pz;
    auto carve = [&](void* base, float** f) {
        Carver c(base);
        f[11] = c.take<float>(n9);         // dmeans2D | dcolors | dopacity | dmeans3D | dcov3D | ddc | dsh | dscales | drot
        f[0] = c.take<float>(Pz);          // opacity (activated)
        f[1] = c.take<float>(3 * Pz);      // scaling
        f[2] = c.take<float>(4 * Pz);      // rotation
        f[12] = c.take<float>(Pz);         // depth
        f[13] = c.take<float>(Pz);         // raw opacity grad
        f[14] = c.take<float>(3 * Pz);     // raw scaling grad
        f[15] = c.take<float>(4 * Pz);     // raw quaternion grad
        f[3] = c.take<float>(n_img);       // raw render
        f[4] = c.take<float>(HW);          // inverse depth
        f[5] = c.take<float>(n_part);      // partial sums
        f[6] = c.take<float>(n_img);       // SSIM map
        f[7] = c.take<float>(n_img);       // dm/dmu1
        f[8] = c.take<float>(n_img);       // dm/dsigma1_sq
        f[9] = c.take<float>(n_img);       // dm/dsigma12
        f[10] = c.take<float>(n_img);      // dL/dimage
        f[16] = reinterpret_cast<float*>(c.take<uint64_t>(1));  // the step's zero-scaling stamp
        return c.off;
    };
    float* f[17];
    const size_t tbytes = carve(nullptr, f);
    void* tbase = alloc(user, DG_BUF_TRAIN, tbytes);
    if (!tbase) return fail("train step scratch allocation failed%s%d");
    carve(tbase, f);
    float *act_o = f[0], *act_s = f[1], *act_q = f[2], *color = f[3], *invd = f[4], *part = f[5];
    float *map = f[6], *dmu1 = f[7], *ds1 = f[8], *ds12 = f[9], *dimg = f[10];
    float* g9 = f[11];
    float *dmeans2D = g9, *dcolors = dmeans2D + 3 * Pz, *dopac = dcolors + 3 * Pz, *dmeans3D = dopac + Pz;
    float *dcov3D = dmeans3D + 3 * Pz, *ddc = dcov3D + 6 * Pz, *dsh = ddc + 3 * Pz, *dscales = dsh + 3 * Mz * Pz;
    float* drot = dscales + 3 * Pz;
    float *depth = f[12], *g_o = f[13], *g_s = f[14], *g_q = f[15];
    // torch's prod backward switches every row to its zero-safe form when any scaling is 0: the activation pass
    // stores this step's stamp when it meets one, and the update compares (no zeroing launch; a fresh 64-bit stamp
    // per step never matches stale memory)
    static std::atomic<uint64_t> step_stamp{0x9e3779b97f4a7c15ull};
    const uint64_t stamp = step_stamp.fetch_add(1, std::memory_order_relaxed) + 1;
    uint64_t* const zstamp = reinterpret_cast<uint64_t*>(f[16]);
    const dg_adam_group* G = a->groups;  // xyz, f_dc, f_rest, opacity, scaling, quaternion
    // Default route: the activations' backward is folded into the update (gmode), and the 4-float chunks that touch
    // no binned row (rcnt == 0: rasterizer gradient exactly zero) skip reading the gradient buffers; the regulariser's
    // partial sums come from the activation launch and the loss from block 0 of the SSIM backward.  Same arithmetic
    // per element as the unfused route (DG_TRAIN_UNFUSED=1: k_activate_bwd, then the plain update; separate loss
    // launches).  (Running the update of those rows on a side stream, overlapping the backward, was measured and
    // dropped: DESIGN.md §8.)
    const bool unfused = getenv("DG_TRAIN_UNFUSED") != nullptr;
    float* const p_sc_fused = part + 3 * nw_ssim;
    // ---- forward: activations, rasterizer, clamp + L1, SSIM.  Default route: the activations (and the regulariser's
    // partial sums) inside the rasterizer's preprocess launch (ActFold); unfused: their own launch.
    if (unfused)
        gs::launch_activate_fwd((uint32_t)P, G[3].param, G[4].param, G[5].param, act_o, act_s, act_q, zstamp, stamp, s);
    // the previous step's overlapped SH update: the emission waits for it (the first launch that reads the SH rows)
    ShOverlap* ov = sh_state(s, a->sh_status != nullptr);
    if (a->sh_status && !ov) return fail("train step: no side stream for the overlapped update%s%d");
    hipEvent_t prev = ov && ov->pending ? ov->done : nullptr;
    if (prev && unfused) { HIP_OK(hipStreamWaitEvent(s, prev, 0)); prev = nullptr; }
    // `pending` stays set until the stream's wait on the previous update is enqueued: on an early error return below
    // the wait is still enqueued (wait_prev), so dg_train_sync / a later step never lose it
    if (ov && !prev) ov->pending = false;
    ActFold fold = {G[3].param, G[4].param, G[5].param, a->loss ? p_sc_fused : nullptr, zstamp, stamp, prev, false};
    auto wait_prev = [&]() {
        if (prev && !fold.waited) (void)hipStreamWaitEvent(s, prev, 0);
        if (ov) ov->pending = false;
    };
    dg_raster_args r = a->view;
    r.means3D = G[0].param; r.dc = G[1].param; r.sh = M > 0 ? G[2].param : nullptr;
    r.opacities = act_o; r.scales = act_s; r.rotations = act_q; r.colors = nullptr; r.cov3D_precomp = nullptr;
    void *geom = nullptr, *binning = nullptr, *image = nullptr, *binning2 = nullptr;
    int64_t num_rendered = 0, num_instances = 0;
    if (forward_impl(&r, color, invd, a->radii, alloc, user, &geom, &binning, &image, &binning2, &num_rendered,
                     &num_instances, stream, nullptr, unfused ? nullptr : &fold)) {
        wait_prev();
        return 1;
    }
    if (prev && !fold.waited) HIP_OK(hipStreamWaitEvent(s, prev, 0));  // nothing was binned: before the backward
    if (ov) ov->pending = false;
    // ---- SparseGaussianAdam.step(radii > 0) over the six groups, ADMM proximal gradient, densification statistics.
    dg_adam_group groups[6];
    const float* grads[6] = {dmeans3D, ddc, dsh, unfused ? g_o : dopac, unfused ? g_s : dscales,
                             unfused ? g_q : drot};
    for (int k = 0; k < 6; k++) {
        groups[k] = G[k];
        groups[k].grad = grads[k];
    }
    if (M <= 0) groups[2].M = 0;  // no rest coefficients: nothing to update
    gs::AdamMultiArgs m;
    memset(&m, 0, sizeof(m));
    m.visible = nullptr; m.vis_radii = a->radii; m.N = (uint32_t)P; m.b1 = 0.9f; m.b2 = 0.999f;
    int n = 0, gk[6];
    for (int k = 0; k < 6; k++) {
        const dg_adam_group& g = groups[k];
        if (g.M == 0) continue;
        if ((uint64_t)P * g.M >= 0xfffff000ull) return fail("train step: group %s%d has N * M >= 2^32", "", k);
        gk[n] = k;
        gs::AdamGroup& d = m.g[n++];
        d.param = g.param; d.grad = g.grad; d.m = g.exp_avg; d.v = g.exp_avg_sq; d.lr = g.lr; d.eps = g.eps; d.M = g.M;
        uintptr_t al = reinterpret_cast<uintptr_t>(g.param) | reinterpret_cast<uintptr_t>(g.grad) |
                       reinterpret_cast<uintptr_t>(g.exp_avg) | reinterpret_cast<uintptr_t>(g.exp_avg_sq);
        if (a->prox[k].u) {
            if (!a->prox[k].z) return fail("train step: group %s%d has prox u without z", "", k);
            d.u = a->prox[k].u; d.z = a->prox[k].z; d.coef = a->prox[k].coef;
            al |= reinterpret_cast<uintptr_t>(a->prox[k].u) | reinterpret_cast<uintptr_t>(a->prox[k].z);
        }
        d.vec = (al & 15u) == 0u;
        if (!unfused && k >= 3) {
            d.gmode = k - 2;  // opacity: sigmoid, scaling: exp + regulariser, quaternion: normalize
            d.act = k == 3 ? act_o : (k == 4 ? act_s : nullptr);
            d.reg = k == 4 ? a->lambda_scale * (1.0f / (float)P) : 0.0f;   // torch's mean backward: x (1 / N)
            if (k == 4) { d.zero_stamp = zstamp; d.stamp = stamp; }
        }
    }
    m.n = n;
    if (a->stats) {
        dg_densify_stats st = *a->stats;
        st.radii = a->radii; st.dmeans2D = dmeans2D; st.dmeans2D_stride = 3;
        if (fill_stats(m, &st)) return 1;
        if (a->depth_threshold > 0.0f) { m.depth = depth; m.depth_thr = a->depth_threshold; }
    }
    if (!unfused) m.hot = carve_geom(geom, P).rcnt;
    const float C1 = 0.01f * 0.01f, C2 = 0.03f * 0.03f;   // fused_ssim's constants
    const float ld = a->lambda_dssim;
    const float g_l1 = (float)(1.0 - (double)ld);
    // loss backward of (1 - ld) L1 + ld (1 - SSIM) + ls mean(prod(scaling)): d/dmap = -ld / n (the mean's backward)
    if (!unfused) {  // render()'s clamp, L1 and the SSIM mean inside the SSIM passes (same values per pixel)
        gs::launch_ssim_fwd_fused(H, W, C1, C2, color, a->gt, a->image, dmu1, ds1, ds12, part, s, a->mask);
        const gs::LossFinal lf = {part, part + nw_ssim, p_sc_fused, nw_ssim, nw_ssim, nb_act, (uint32_t)n_img,
                                  (uint32_t)P, a->loss, a->mask ? part + 2 * nw_ssim : nullptr, nw_ssim};
        // d/dmask of lambda_mask mean((mask - 1)^2): (lambda_mask (1 / n)) (2 (mask - 1)), as torch's mean backward
        // (a multiply by the float reciprocal) and pow's backward form it; the factor 2 is exact
        const float mreg = 2.0f * (a->lambda_mask * (1.0f / (float)n_img));
        gs::launch_ssim_bwd_fused(H, W, a->image, a->gt, color, (-ld) / (float)n_img, g_l1 / (float)n_img, dmu1, ds1,
                                  ds12, dimg, s, a->loss ? &lf : nullptr, a->mask, a->dmask, mreg);
    } else {
        gs::launch_clamp_l1_fwd((uint32_t)n_img, color, a->gt, a->image, part, s);
        gs::launch_ssim_fwd(1, 3, H, W, C1, C2, a->image, a->gt, map, dmu1, ds1, ds12, s);
        if (a->loss) {
            gs::launch_block_sum(map, (uint32_t)n_img, 0, part + nb_l1, s);
            gs::launch_block_sum(act_s, (uint32_t)P, 1, part + nb_l1 + nb_map, s);
            gs::launch_loss_final(part, nb_l1, part + nb_l1, nb_map, part + nb_l1 + nb_map, nb_sc, (uint32_t)n_img,
                                  (uint32_t)P, a->loss, s);
        }
        gs::launch_ssim_bwd(1, 3, H, W, a->image, a->gt, nullptr, dmu1, ds1, ds12, map, s, (-ld) / (float)n_img);
        gs::launch_clamp_l1_bwd((uint32_t)n_img, color, a->image, a->gt, map, nullptr, dimg, s, g_l1);
    }
    if (dg_rasterize_backward(&r, a->radii, geom, binning, image, binning2, num_rendered, num_instances, dimg, nullptr,
                              dmeans2D, dcolors, dopac, dmeans3D, dcov3D, ddc, dsh, dscales, drot, depth, alloc, user,
                              stream))
        return 1;
    if (unfused)
        gs::launch_activate_bwd((uint32_t)P, act_o, act_s, G[5].param, dopac, dscales, drot, g_o, g_s, g_q, s,
                                a->lambda_scale * (1.0f / (float)P), zstamp, stamp);
#ifndef DG_DIAG_NO_ADAM  // timing diagnostic only (no parameter update): what the update costs the next step's forward
    if (a->sh_status) {
        // xyz / opacity / scaling / rotation + statistics + the rows' status snapshot here (the next forward's
        // preprocess reads them); f_dc / f_rest (81% of the bytes) on the side stream from the snapshot, overlapping
        // the next step's forward until its emission (the launches in between read neither them nor the snapshot)
        gs::AdamMultiArgs mg = m, ms = m;
        mg.n = ms.n = 0;
        for (int i = 0; i < n; i++) {
            if (gk[i] == 1 || gk[i] == 2) ms.g[ms.n++] = m.g[i];
            else mg.g[mg.n++] = m.g[i];
        }
        mg.status_out = a->sh_status;
        ms.status = a->sh_status;
        ms.radii = nullptr;  // no statistics on the side
        ms.grid_cap = sh_grid_cap();
        gs::launch_adam_multi(mg, s);
        HIP_OK(hipEventRecord(ov->fork, s));
        HIP_OK(hipStreamWaitEvent(ov->side, ov->fork, 0));
        if (ms.n) gs::launch_adam_multi(ms, ov->side);
        HIP_OK(hipEventRecord(ov->done, ov->side));
        ov->pending = true;
    } else {
        gs::launch_adam_multi(m, s);
    }
#endif
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_train_sync(dg_stream_t stream) {
    API_GUARD();
    ShOverlap* ov = sh_state((hipStream_t)stream, false);
    if (ov && ov->pending) {
        HIP_OK(hipStreamWaitEvent((hipStream_t)stream, ov->done, 0));
        ov->pending = false;
    }
    return 0;
}

int dg_add_densification_stats(const dg_densify_stats* stats, const uint8_t* visible, uint32_t N, dg_stream_t stream) {
    if (!stats) return fail("stats required%s%d");
    return dg_adam_update_groups(nullptr, 0, visible, N, 0.9f, 0.999f, stats, stream);
}

namespace {
struct DensifyState {  // DG_BUF_DENSIFY: selection of the N originals
    uint32_t *clone_flag, *split_flag, *clone_pos, *split_pos, *clone_idx, *split_idx, *totals;
    void* scan_tmp;
    size_t bytes;
};
DensifyState carve_densify(void* base, uint32_t N) {
    Carver c(base);
    DensifyState d;
    const size_t n = N ? N : 1;
    d.clone_flag = c.take<uint32_t>(n); d.split_flag = c.take<uint32_t>(n);
    d.clone_pos = c.take<uint32_t>(n); d.split_pos = c.take<uint32_t>(n);
    d.clone_idx = c.take<uint32_t>(n); d.split_idx = c.take<uint32_t>(n);
    d.totals = c.take<uint32_t>(4);
    d.scan_tmp = c.take<char>(gs::scan_temp_bytes((uint32_t)n));
    d.bytes = c.off;
    return d;
}
struct KeepState {  // DG_BUF_DENSIFY2: the C candidate rows
    uint32_t *keep, *keep_pos, *total;
    void* scan_tmp;
    size_t bytes;
};
KeepState carve_keep(void* base, uint64_t C) {
    Carver c(base);
    KeepState k;
    const size_t n = C ? (size_t)C : 1;
    k.keep = c.take<uint32_t>(n); k.keep_pos = c.take<uint32_t>(n); k.total = c.take<uint32_t>(4);
    k.scan_tmp = c.take<char>(gs::scan_temp_bytes((uint32_t)n));
    k.bytes = c.off;
    return k;
}
int densify_check(const dg_densify_args* a, bool need_stats = true) {
    if (!a) return fail("null densify args%s%d");
    const dg_gaussian_set& g = a->set;
    for (int q = 0; q < 6; q++) {
        if (g.N && !g.params[q]) return fail("parameter tensor %s%d is NULL", "", q);
        if ((g.exp_avg[q] == nullptr) != (g.exp_avg_sq[q] == nullptr))
            return fail("exp_avg / exp_avg_sq of tensor %s%d: both or neither", "", q);
    }
    if (g.width[0] != 3 || g.width[4] != 3 || g.width[5] != 4 || g.width[3] != 1)
        return fail("widths must be xyz 3, opacity 1, scaling 3, quaternion 4%s%d");
    if (need_stats && g.N && (!g.grad_accum || !g.denom)) return fail("grad_accum and denom required%s%d");
    return 0;
}
gs::DensifyArgs densify_args(const dg_densify_args* a, const DensifyState& st) {
    gs::DensifyArgs d;
    memset(&d, 0, sizeof(d));
    const dg_gaussian_set& g = a->set;
    d.N = g.N;
    d.xyz = g.params[0]; d.f_dc = g.params[1]; d.f_rest = g.params[2]; d.opacity = g.params[3];
    d.scaling = g.params[4]; d.rot = g.params[5];
    for (int q = 0; q < 6; q++) { d.m[q] = g.exp_avg[q]; d.v[q] = g.exp_avg_sq[q]; d.width[q] = g.width[q]; }
    d.grad_accum = g.grad_accum; d.denom = g.denom;
    d.grad_threshold = a->max_grad; d.dense_extent = a->dense_extent;
    d.clone_flag = st.clone_flag; d.split_flag = st.split_flag;
    return d;
}
}  // namespace

int dg_densify_select(dg_densify_args* a, dg_alloc_fn alloc, void* user, dg_stream_t stream) {
    if (densify_check(a)) return 1;
    hipStream_t s = (hipStream_t)stream;
    const uint32_t N = a->set.N;
    a->nc = a->ns = a->n_out = 0;
    a->state = alloc(user, DG_BUF_DENSIFY, carve_densify(nullptr, N).bytes);
    if (!a->state) return fail("densify state allocation failed%s%d");
    a->state2 = nullptr;
    if (N == 0) return 0;
    DensifyState st = carve_densify(a->state, N);
    gs::DensifyArgs d = densify_args(a, st);
    gs::launch_densify_select(d, s);
    gs::exclusive_scan(st.clone_flag, N, st.clone_pos, st.totals, st.scan_tmp, s);
    gs::exclusive_scan(st.split_flag, N, st.split_pos, st.totals + 1, st.scan_tmp, s);
    gs::launch_densify_lists(d, st.clone_pos, st.split_pos, st.clone_idx, st.split_idx, s);
    uint32_t h[2];
    HIP_OK(hipMemcpyAsync(h, st.totals, sizeof(h), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    a->nc = h[0];
    a->ns = h[1];
    HIP_OK(hipGetLastError());
    return 0;
}

namespace {
__global__ void k_split_stds(const uint32_t* __restrict__ split_idx, uint32_t ns, uint32_t replicas,
                             const float* __restrict__ scaling, float* __restrict__ stds) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= 3u * ns * replicas) return;
    const uint32_t row = t / 3u, c = t % 3u;
    stds[t] = expf(scaling[3 * (size_t)split_idx[row % ns] + c]);
}
}  // namespace

int dg_densify_split_stds(const dg_densify_args* a, float* stds, dg_stream_t stream) {
    if (!a || !a->state) return fail("dg_densify_select first%s%d");
    if (a->ns == 0) return 0;
    const uint32_t r = a->replicas ? a->replicas : 2;
    DensifyState st = carve_densify(a->state, a->set.N);
    const uint32_t n = 3u * a->ns * r;
    k_split_stds<<<(n + 255) / 256, 256, 0, (hipStream_t)stream>>>(st.split_idx, a->ns, r, a->set.params[4], stds);
    HIP_OK(hipGetLastError());
    return 0;
}

namespace {
gs::RebuildArgs rebuild_args(const dg_densify_args* a, const DensifyState& st, const KeepState& ks) {
    gs::RebuildArgs r;
    memset(&r, 0, sizeof(r));
    r.d = densify_args(a, st);
    r.nc = a->nc; r.ns = a->ns; r.replicas = a->replicas ? a->replicas : 2;
    r.clone_idx = st.clone_idx; r.split_idx = st.split_idx; r.samples = a->samples;
    r.min_opacity = a->min_opacity; r.use_bbox = a->use_bbox; r.bbox_z = a->bbox_z;
    r.use_screen = a->use_screen; r.max_screen = a->max_screen_size; r.big_extent = a->big_extent;
    r.keep = ks.keep;
    for (int q = 0; q < 6; q++) { r.out_p[q] = a->out_params[q]; r.out_m[q] = a->out_exp_avg[q]; r.out_v[q] = a->out_exp_avg_sq[q]; }
    return r;
}
}  // namespace

int dg_densify_count(dg_densify_args* a, dg_alloc_fn alloc, void* user, dg_stream_t stream) {
    if (densify_check(a)) return 1;
    if (!a->state) return fail("dg_densify_select first%s%d");
    if (a->ns && !a->samples) return fail("samples [replicas*ns, 3] required%s%d");
    hipStream_t s = (hipStream_t)stream;
    const uint32_t r = a->replicas ? a->replicas : 2;
    const uint64_t C = (uint64_t)a->set.N + a->nc + (uint64_t)r * a->ns;
    uint64_t wsum = 0;
    for (int q = 0; q < 6; q++) wsum += a->set.width[q];
    if (C * wsum >= 0xfffff000ull) return fail("too many candidate rows x floats%s%d");
    a->state2 = alloc(user, DG_BUF_DENSIFY2, carve_keep(nullptr, C).bytes);
    if (!a->state2) return fail("densify candidate allocation failed%s%d");
    a->n_out = 0;
    if (C == 0) return 0;
    DensifyState st = carve_densify(a->state, a->set.N);
    KeepState ks = carve_keep(a->state2, C);
    gs::RebuildArgs rb = rebuild_args(a, st, ks);
    gs::launch_densify_keep(rb, s);
    gs::exclusive_scan(ks.keep, (uint32_t)C, ks.keep_pos, ks.total, ks.scan_tmp, s);
    uint32_t h = 0;
    HIP_OK(hipMemcpyAsync(&h, ks.total, sizeof(h), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    a->n_out = h;
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_densify_gather(const dg_densify_args* a, dg_stream_t stream) {
    if (densify_check(a, false)) return 1;
    if (!a->state || !a->state2) return fail("dg_densify_select and dg_densify_count first%s%d");
    for (int q = 0; q < 6; q++) {
        if (a->n_out && !a->out_params[q]) return fail("output tensor %s%d is NULL", "", q);
        if ((a->out_exp_avg[q] == nullptr) != (a->out_exp_avg_sq[q] == nullptr))
            return fail("output moments of tensor %s%d: both or neither", "", q);
    }
    if (a->n_out == 0) return 0;
    const uint32_t r = a->replicas ? a->replicas : 2;
    const uint64_t C = (uint64_t)a->set.N + a->nc + (uint64_t)r * a->ns;
    DensifyState st = carve_densify(a->state, a->set.N);
    KeepState ks = carve_keep(a->state2, C);
    gs::RebuildArgs rb = rebuild_args(a, st, ks);
    gs::launch_densify_gather(rb, ks.keep_pos, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

namespace {
__global__ void __launch_bounds__(256) k_keep_from_mask(const uint8_t* __restrict__ prune, uint32_t N,
                                                        uint32_t* __restrict__ keep) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < N) keep[i] = prune[i] ? 0u : 1u;
}
__global__ void __launch_bounds__(256) k_gather_stats(const uint32_t* __restrict__ keep,
                                                      const uint32_t* __restrict__ keep_pos, uint32_t N,
                                                      const float* __restrict__ ga, const float* __restrict__ dn,
                                                      const float* __restrict__ mr, float* __restrict__ oga,
                                                      float* __restrict__ odn, float* __restrict__ omr) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= N || !keep[i]) return;
    const uint32_t o = keep_pos[i];
    if (oga) oga[o] = ga[i];
    if (odn) odn[o] = dn[i];
    if (omr) omr[o] = mr[i];
}
}  // namespace

int dg_prune_select(dg_densify_args* a, const uint8_t* prune_mask, dg_alloc_fn alloc, void* user,
                    dg_stream_t stream) {
    if (!a) return fail("null densify args%s%d");
    const dg_gaussian_set& g = a->set;
    for (int q = 0; q < 6; q++) {
        if (g.N && !g.params[q]) return fail("parameter tensor %s%d is NULL", "", q);
        if ((g.exp_avg[q] == nullptr) != (g.exp_avg_sq[q] == nullptr))
            return fail("exp_avg / exp_avg_sq of tensor %s%d: both or neither", "", q);
    }
    if (g.width[0] != 3 || g.width[4] != 3 || g.width[5] != 4 || g.width[3] != 1)
        return fail("widths must be xyz 3, opacity 1, scaling 3, quaternion 4%s%d");
    if (g.N && !prune_mask) return fail("prune mask required%s%d");
    uint64_t wsum = 0;
    for (int q = 0; q < 6; q++) wsum += g.width[q];
    if ((uint64_t)g.N * wsum >= 0xfffff000ull) return fail("too many rows x floats%s%d");
    hipStream_t s = (hipStream_t)stream;
    const uint32_t N = g.N;
    a->nc = a->ns = a->n_out = 0;
    a->samples = nullptr;
    a->state = alloc(user, DG_BUF_DENSIFY, carve_densify(nullptr, N).bytes);
    a->state2 = alloc(user, DG_BUF_DENSIFY2, carve_keep(nullptr, N).bytes);
    if (!a->state || !a->state2) return fail("prune state allocation failed%s%d");
    if (N == 0) return 0;
    KeepState ks = carve_keep(a->state2, N);
    k_keep_from_mask<<<(N + 255) / 256, 256, 0, s>>>(prune_mask, N, ks.keep);
    gs::exclusive_scan(ks.keep, N, ks.keep_pos, ks.total, ks.scan_tmp, s);
    uint32_t h = 0;
    HIP_OK(hipMemcpyAsync(&h, ks.total, sizeof(h), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    a->n_out = h;
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_prune_gather_stats(const dg_densify_args* a, const float* max_radii2D, float* out_grad_accum,
                          float* out_denom, float* out_max_radii2D, dg_stream_t stream) {
    if (!a || !a->state2) return fail("dg_prune_select first%s%d");
    if (a->nc || a->ns) return fail("statistics are gathered for a pure prune only%s%d");
    const uint32_t N = a->set.N;
    if (N == 0 || a->n_out == 0) return 0;
    if ((out_grad_accum && !a->set.grad_accum) || (out_denom && !a->set.denom) || (out_max_radii2D && !max_radii2D))
        return fail("a statistics source is NULL%s%d");
    KeepState ks = carve_keep(a->state2, N);
    k_gather_stats<<<(N + 255) / 256, 256, 0, (hipStream_t)stream>>>(ks.keep, ks.keep_pos, N, a->set.grad_accum,
                                                                    a->set.denom, max_radii2D, out_grad_accum,
                                                                    out_denom, out_max_radii2D);
    HIP_OK(hipGetLastError());
    return 0;
}

uint32_t dg_clamp_l1_blocks(uint32_t n) { return gs::clamp_l1_blocks(n); }

int dg_clamp_l1_forward(uint32_t n, const float* img, const float* gt, float* clamped, float* partial,
                        dg_stream_t stream) {
    if (n == 0) return 0;
    if (!img || !gt || !clamped || !partial) return fail("clamp_l1: NULL tensor%s%d");
    if ((reinterpret_cast<uintptr_t>(img) | reinterpret_cast<uintptr_t>(gt) | reinterpret_cast<uintptr_t>(clamped)) & 15u)
        return fail("clamp_l1: tensors must be 16-byte aligned%s%d");
    gs::launch_clamp_l1_fwd(n, img, gt, clamped, partial, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_clamp_l1_backward(uint32_t n, const float* img, const float* clamped, const float* gt, const float* g_clamped,
                         const float* g_l1, float* d_img, dg_stream_t stream) {
    if (n == 0) return 0;
    if (!img || !gt || !d_img) return fail("clamp_l1 backward: NULL tensor%s%d");  // clamped: recomputed, may be NULL
    gs::launch_clamp_l1_bwd(n, img, clamped, gt, g_clamped, g_l1, d_img, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_row_prod_forward(uint32_t N, uint32_t M, const float* x, float* prod, uint32_t* zero_stamp, uint32_t stamp,
                        dg_stream_t stream) {
    if (M < 1 || M > 3) return fail("row_prod: 1 <= M <= 3 columns%s%d");
    if (!zero_stamp || (N && (!x || !prod))) return fail("row_prod: NULL tensor%s%d");
    gs::launch_row_prod_fwd(N, M, x, prod, zero_stamp, stamp, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_row_prod_backward(uint32_t N, uint32_t M, const float* x, const float* prod, const float* dprod,
                         const uint32_t* zero_stamp, uint32_t stamp, float* dx, dg_stream_t stream) {
    if (M < 1 || M > 3) return fail("row_prod backward: 1 <= M <= 3 columns%s%d");
    if (N == 0) return 0;
    if (!x || !prod || !dprod || !zero_stamp || !dx) return fail("row_prod backward: NULL tensor%s%d");
    gs::launch_row_prod_bwd(N, M, x, prod, dprod, zero_stamp, stamp, dx, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_activate_forward(uint32_t N, const float* raw_opacity, const float* raw_scaling, const float* raw_rotation,
                        float* opacity, float* scaling, float* rotation, dg_stream_t stream) {
    if (N == 0) return 0;
    if (!raw_opacity || !raw_scaling || !raw_rotation || !opacity || !scaling || !rotation)
        return fail("activate: NULL tensor%s%d");
    if ((reinterpret_cast<uintptr_t>(raw_rotation) | reinterpret_cast<uintptr_t>(rotation)) & 15u)
        return fail("activate: rotation rows must be 16-byte aligned%s%d");
    gs::launch_activate_fwd(N, raw_opacity, raw_scaling, raw_rotation, opacity, scaling, rotation, nullptr, 0,
                            (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_activate_backward(uint32_t N, const float* opacity, const float* scaling, const float* raw_rotation,
                         const float* d_opacity, const float* d_scaling, const float* d_rotation, float* d_raw_opacity,
                         float* d_raw_scaling, float* d_raw_rotation, dg_stream_t stream) {
    if (N == 0) return 0;
    if (!opacity || !scaling || !raw_rotation || !d_raw_opacity || !d_raw_scaling || !d_raw_rotation)
        return fail("activate backward: NULL tensor%s%d");
    if ((reinterpret_cast<uintptr_t>(raw_rotation) | reinterpret_cast<uintptr_t>(d_raw_rotation) |
         reinterpret_cast<uintptr_t>(d_rotation)) & 15u)
        return fail("activate backward: rotation rows must be 16-byte aligned%s%d");
    gs::launch_activate_bwd(N, opacity, scaling, raw_rotation, d_opacity, d_scaling, d_rotation, d_raw_opacity,
                            d_raw_scaling, d_raw_rotation, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_splat_pack(uint32_t N, const float* xyz, const float* scaling, const float* opacity, const float* rotation,
                  const float* f_dc, uint8_t* out, dg_alloc_fn alloc, void* user, dg_stream_t stream) {
    if (N == 0) return 0;
    if (!xyz || !scaling || !opacity || !rotation || !f_dc || !out) return fail("splat pack: NULL tensor%s%d");
    hipStream_t s = (hipStream_t)stream;
    Carver c(nullptr);
    c.take<uint32_t>(N); c.take<uint32_t>(N); c.take<uint32_t>(N); c.take<uint32_t>(N);
    c.take<char>(gs::radix_sort_temp_bytes(N));
    void* base = alloc(user, DG_BUF_TEMP, c.off);
    if (!base) return fail("splat pack scratch allocation failed%s%d");
    Carver d(base);
    uint32_t* k0 = d.take<uint32_t>(N);
    uint32_t* v0 = d.take<uint32_t>(N);
    uint32_t* k1 = d.take<uint32_t>(N);
    uint32_t* v1 = d.take<uint32_t>(N);
    void* tmp = d.take<char>(gs::radix_sort_temp_bytes(N));
    gs::launch_splat_keys(N, scaling, opacity, k0, v0, s);
    const int which = gs::radix_sort_pairs(k0, v0, k1, v1, nullptr, N, 0, 32, tmp, s);  // stable: ties by index
    gs::launch_splat_pack(N, which ? v1 : v0, xyz, scaling, opacity, rotation, f_dc, out, s);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_ply_pack(uint32_t N, const float* xyz, const float* f_dc, uint8_t* out, dg_stream_t stream) {
    if (N == 0) return 0;
    if (!xyz || !f_dc || !out) return fail("ply pack: NULL tensor%s%d");
    gs::launch_ply_pack(N, xyz, f_dc, out, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_points_in_boxes2d(uint32_t N, const double* points, uint32_t stride, const dg_box2d_set* boxes,
                         uint8_t* labels, double* transformed, uint32_t* counts, int want_members, dg_alloc_fn alloc,
                         void* user, dg_stream_t stream) {
    static_assert(DG_MAX_BOXES == gs::BOX_MAX, "box capacity");
    if (!boxes || boxes->C == 0 || boxes->C > DG_MAX_BOXES) return fail("points_in_boxes2d: 1..%s%d boxes", "", DG_MAX_BOXES);
    if (!counts) return fail("points_in_boxes2d: NULL counts%s%d");
    const uint32_t C = boxes->C;
    for (uint32_t k = 0; k < C; k++) counts[k] = 0;
    if (N == 0) return 0;
    if (!points || stride < 2) return fail("points_in_boxes2d: NULL points or stride < 2%s%d");
    if (!alloc) return fail("points_in_boxes2d: NULL allocator%s%d");
    hipStream_t s = (hipStream_t)stream;
    const uint32_t nb = gs::box_blocks(N);
    Carver c(nullptr);
    c.take<uint64_t>(N); c.take<uint32_t>((size_t)C * nb); c.take<uint32_t>(C);
    void* base = alloc(user, DG_BUF_TEMP, c.off);
    if (!base) return fail("points_in_boxes2d scratch allocation failed%s%d");
    Carver d(base);
    uint64_t* masks = d.take<uint64_t>(N);
    uint32_t* cnt = d.take<uint32_t>((size_t)C * nb);
    uint32_t* total = d.take<uint32_t>(C);
    gs::BoxSet bs;
    bs.C = C;
    bs.has_T = boxes->has_T;
    for (int q = 0; q < 6; q++) bs.T[q] = boxes->T[q];
    for (uint32_t k = 0; k < gs::BOX_MAX; k++)
        for (int q = 0; q < 4; q++) bs.box[k][q] = k < C ? boxes->box[k][q] : 0.0;
    gs::launch_box_test(N, points, stride, bs, labels, transformed, masks, cnt, s);
    gs::launch_box_scan(N, C, cnt, total, s);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(counts, total, C * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    if (!want_members) return 0;
    gs::BoxOffsets off;
    off.C = C;
    uint64_t run = 0;
    for (uint32_t k = 0; k < gs::BOX_MAX; k++) {
        off.first[k] = (uint32_t)run;
        if (k < C) run += counts[k];
    }
    if (run > 0xffffffffull) return fail("points_in_boxes2d: %s%d members exceed 2^32", "", 0);
    uint32_t* members = (uint32_t*)alloc(user, DG_BUF_MEMBERS, run * sizeof(uint32_t));
    if (!members) return fail("points_in_boxes2d member allocation failed%s%d");
    gs::launch_box_scatter(N, masks, cnt, off, members, s);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_adam_update(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, const uint8_t* visible,
                   float lr, float b1, float b2, float eps, uint32_t N, uint32_t M, dg_stream_t stream) {
    gs::launch_adam(param, grad, exp_avg, exp_avg_sq, (const bool*)visible, lr, b1, b2, eps, N, M, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_fused_ssim_forward(int B, int CH, int H, int W, float C1, float C2, const float* img1, const float* img2,
                          float* ssim_map, float* dm_dmu1, float* dm_dsigma1_sq, float* dm_dsigma12,
                          dg_stream_t stream) {
    if (dm_dmu1 && (!dm_dsigma1_sq || !dm_dsigma12)) return fail("train=True needs all three partial maps%s%d");
    gs::launch_ssim_fwd(B, CH, H, W, C1, C2, img1, img2, ssim_map, dm_dmu1, dm_dsigma1_sq, dm_dsigma12,
                        (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_fused_ssim_backward(int B, int CH, int H, int W, float C1, float C2, const float* img1, const float* img2,
                           const float* dL_dmap, const float* dm_dmu1, const float* dm_dsigma1_sq,
                           const float* dm_dsigma12, float* dL_dimg1, dg_stream_t stream) {
    (void)C1; (void)C2;
    gs::launch_ssim_bwd(B, CH, H, W, img1, img2, dL_dmap, dm_dmu1, dm_dsigma1_sq, dm_dsigma12, dL_dimg1,
                        (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

uint32_t dg_fused_ssim_parts(int B, int CH, int H, int W) {
    if (B <= 0 || CH <= 0 || H <= 0 || W <= 0) return 1u;
    const uint32_t n = gs::ssim_mean_parts(B, CH, H, W);
    return n ? n : 1u;
}

int dg_fused_ssim_mean(int B, int CH, int H, int W, float C1, float C2, const float* img1, const float* img2,
                       float* dm_dmu1, float* dm_dsigma1_sq, float* dm_dsigma12, float* part, float* mean,
                       dg_stream_t stream) {
    if (B < 0 || CH < 0 || H < 0 || W < 0) return fail("fused_ssim mean: negative size%s%d");
    if ((size_t)B * CH * H * W >= 0xffffff00ull) return fail("fused_ssim mean: image too large%s%d");
    if (!part || !mean) return fail("fused_ssim mean: NULL partials or output%s%d");
    if (dm_dmu1 && (!dm_dsigma1_sq || !dm_dsigma12)) return fail("train=True needs all three partial maps%s%d");
    if ((size_t)B * CH * H * W && (!img1 || !img2)) return fail("fused_ssim mean: NULL image%s%d");
    gs::launch_ssim_mean(B, CH, H, W, C1, C2, img1, img2, dm_dmu1, dm_dsigma1_sq, dm_dsigma12, part, mean,
                         (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_fused_ssim_mean_backward(int B, int CH, int H, int W, const float* img1, const float* img2,
                                const float* dL_dmean, const float* dm_dmu1, const float* dm_dsigma1_sq,
                                const float* dm_dsigma12, float* dL_dimg1, dg_stream_t stream) {
    if ((size_t)B * CH * H * W == 0) return 0;
    if ((size_t)B * CH * H * W >= 0xffffff00ull) return fail("fused_ssim mean backward: image too large%s%d");
    if (!img1 || !img2 || !dL_dmean || !dm_dmu1 || !dm_dsigma1_sq || !dm_dsigma12 || !dL_dimg1)
        return fail("fused_ssim mean backward: NULL tensor%s%d");
    gs::launch_ssim_mean_bwd(B, CH, H, W, img1, img2, dL_dmean, dm_dmu1, dm_dsigma1_sq, dm_dsigma12, dL_dimg1,
                             (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_mean_of_parts(const float* part, uint32_t n_part, uint32_t denom, float* out, dg_stream_t stream) {
    if (!out || (n_part && !part)) return fail("mean_of_parts: NULL tensor%s%d");
    gs::launch_mean_parts(part, n_part, denom, out, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_dist_cuda2(int P, const float* points, float* out, dg_alloc_fn alloc, void* user, dg_stream_t stream) {
    if (P <= 0) return 0;
    void* t = alloc(user, DG_BUF_TEMP, gs::knn_temp_bytes(P));
    if (!t) return fail("knn scratch allocation failed%s%d");
    gs::launch_knn(P, points, out, t, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
    return 0;
}

namespace {
__global__ void k_gather_g(uint32_t K, const uint32_t* s_e, const uint32_t* eg, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < K) out[i] = eg[s_e[i]];
}
// tile id of every binned position: out[i] = t for i in ranges[t] (tiles with only[t] == 0 skipped)
__global__ void k_tiles_of(int T, const uint2* ranges, const uint8_t* only, uint32_t* out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T || (only && !only[t])) return;
    const uint2 r = ranges[t];
    for (uint32_t i = r.x; i < r.y; i++) out[i] = (uint32_t)t;
}
}  // namespace

int dg_debug_sorted_instances(const dg_raster_args* a, const void* geom, const void* binning, const void* binning2,
                              const void* image, int64_t num_rendered, int64_t num_instances, uint32_t* tiles_out,
                              uint32_t* gauss_out, int64_t* e1_out, dg_stream_t stream) {
    hipStream_t s = (hipStream_t)stream;
    const int T = tiles_x_of(a->W) * tiles_y_of(a->H);
    Geom g = carve_geom((void*)geom, a->P);
    Image im = carve_image((void*)image, a->W, a->H);
    uint32_t hc[16];
    HIP_OK(hipMemcpyAsync(hc, g.counters, sizeof(hc), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    const uint32_t E1 = hc[gs::CNT_E1];
    *e1_out = E1;
    const int64_t Kcap = inst_cap((uint64_t)num_rendered);
    if (E1 > 0) {
        Binning b = carve_binning((void*)binning, num_instances);
        k_gather_g<<<(E1 + 255) / 256, 256, 0, s>>>(E1, b.se, b.eg, gauss_out);
        k_tiles_of<<<(T + 255) / 256, 256, 0, s>>>(T, im.ranges, nullptr, tiles_out);
    }
    const int64_t K2 = binning2 ? (int64_t)hc[gs::CNT_K2] : 0;
    if (binning2 && K2 > 0) {
        Binning b2 = carve_binning((void*)binning2, Kcap);
        k_gather_g<<<(unsigned)((K2 + 255) / 256), 256, 0, s>>>((uint32_t)K2, b2.se, b2.eg, gauss_out + E1);
        k_tiles_of<<<(T + 255) / 256, 256, 0, s>>>(T, im.ranges2, im.unfinished, tiles_out + E1);
    }
    HIP_OK(hipGetLastError());
    return 0;
}

int dg_binned_instances(const void* geom, int P, int64_t* binned, dg_stream_t stream) {
    hipStream_t s = (hipStream_t)stream;
    Geom g = carve_geom((void*)geom, P);
    uint32_t hc[16];
    HIP_OK(hipMemcpyAsync(hc, g.counters, sizeof(hc), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    *binned = (int64_t)hc[gs::CNT_E1] + (int64_t)hc[gs::CNT_K2];
    return 0;
}

int dg_debug_counters(const void* geom, int P, uint32_t* counters16, dg_stream_t stream) {
    hipStream_t s = (hipStream_t)stream;
    Geom g = carve_geom((void*)geom, P);
    HIP_OK(hipMemcpyAsync(counters16, g.counters, 16 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    return 0;
}

int dg_debug_geometry(const void* geom, int P, float* means2D, float* conic_opacity, float* rgb_invdepth,
                      uint32_t* tile_count, dg_stream_t stream) {
    if (P <= 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    Geom g = carve_geom((void*)geom, P);
    if (means2D) HIP_OK(hipMemcpy2DAsync(means2D, 8, g.sp, 32, 8, (size_t)P, hipMemcpyDeviceToDevice, s));
    if (conic_opacity)
        HIP_OK(hipMemcpy2DAsync(conic_opacity, 16, (const char*)g.sp + 8, 32, 16, (size_t)P, hipMemcpyDeviceToDevice, s));
    if (rgb_invdepth) HIP_OK(hipMemcpyAsync(rgb_invdepth, g.rgbi, 16 * (size_t)P, hipMemcpyDeviceToDevice, s));
    if (tile_count) HIP_OK(hipMemcpyAsync(tile_count, g.rcnt, 4 * (size_t)P, hipMemcpyDeviceToDevice, s));
    return 0;
}

int dg_debug_image_state(const void* image, int W, int H, float* final_T, uint32_t* n_contrib, uint32_t* max_contrib,
                         uint32_t* ranges, dg_stream_t stream) {
    hipStream_t s = (hipStream_t)stream;
    Image im = carve_image((void*)image, W, H);
    const size_t HW = (size_t)W * H, T = (size_t)tiles_x_of(W) * tiles_y_of(H);
    if (final_T) HIP_OK(hipMemcpyAsync(final_T, im.final_T, 4 * HW, hipMemcpyDeviceToDevice, s));
    if (n_contrib) HIP_OK(hipMemcpyAsync(n_contrib, im.n_contrib, 4 * HW, hipMemcpyDeviceToDevice, s));
    if (max_contrib) HIP_OK(hipMemcpyAsync(max_contrib, im.max_contrib, 4 * T, hipMemcpyDeviceToDevice, s));
    if (ranges) HIP_OK(hipMemcpyAsync(ranges, im.ranges, 8 * T, hipMemcpyDeviceToDevice, s));
    return 0;
}

int dg_shutdown(void) {
    // new calls fail from here on; wait (bounded) for the calls already inside the library to leave
    g_shutting_down.store(true, std::memory_order_release);
    for (int i = 0; i < 5000 && g_calls_in_flight.load(std::memory_order_acquire) > 0; i++)
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    if (g_calls_in_flight.load(std::memory_order_acquire) > 0) return fail("shutdown: calls still in flight%s%d");
    // side streams of the overlapped SH update: drain, then destroy (with their events)
    {
        std::lock_guard<std::mutex> lk(sh_mu());
        for (auto& kv : sh_map()) {
            ShOverlap& o = kv.second;
            if (o.side) { (void)hipStreamSynchronize(o.side); (void)hipStreamDestroy(o.side); }
            if (o.fork) (void)hipEventDestroy(o.fork);
            if (o.done) (void)hipEventDestroy(o.done);
        }
        sh_map().clear();
    }
    {
        std::lock_guard<std::mutex> lk(g_cap_mu);
        for (auto& kv : cap_probes())
            if (kv.second.probe) (void)hipFree(kv.second.probe);
        cap_probes().clear();
        drain_cap_graveyard_locked();
    }
    {
        auto release = [](HostCounters& h) {
            if (h.ev) (void)hipEventDestroy(h.ev);
            if (h.buf) (void)hipHostFree(h.buf);
            h = HostCounters();
        };
        release(host_counters_slot().h);  // this thread's; other threads return theirs to the pool on exit
        std::lock_guard<std::mutex> lk(hc_mu());
        for (auto& h : hc_pool()) release(h);
        hc_pool().clear();
    }
    for (auto& r : g_prof_recs) { g_ev_pool.push_back(r.a); g_ev_pool.push_back(r.b); }
    g_prof_recs.clear();
    for (hipEvent_t e : g_ev_pool) (void)hipEventDestroy(e);
    g_ev_pool.clear();
    g_prof = false;
    return 0;
}

}  // extern "C"
