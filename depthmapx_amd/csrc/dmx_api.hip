// dmx_api.hip -- implementation of the C ABI in include/dmx.h (unity build with the kernels).
//
// Host orchestration only: uploads the point map (SoA in HBM), launches the HIP kernels on the
// context stream, sizes/retries scratch, and copies results out in reference layout.  There is no
// CPU implementation of the sweep or the BFS behind this ABI: if the GPU path cannot run, the call
// fails with a status code.
#include <hip/hip_runtime.h>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dmx.h"
#include "policy.hpp"
#include "host/graphfile.hpp"
#include "host/graphio.hpp"
#include "host/pointmap.hpp"
#include "kernels/makegraph.hip"
#include "kernels/vga.hip"
#include "kernels/vga_do.hip"
#include "kernels/vga_tile.hip"
#include "kernels/stepdepth.hip"
#include "kernels/vga_local.hip"
#include "kernels/fill.hip"
#include "kernels/vstep.hip"
#include "kernels/vga_ordered.hip"

using namespace dmx;

namespace {
thread_local std::string g_err;
double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
bool verbose() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("DMX_VERBOSE");
        v = (e && *e && strcmp(e, "0") != 0) ? 1 : 0;
    }
    return v == 1;
}
#define VLOG(...)                                      \
    do {                                               \
        if (verbose()) fprintf(stderr, "[dmx] " __VA_ARGS__); \
    } while (0)
// Every host<->device copy is ordered on the context's (non-blocking) stream: a plain hipMemcpy
// runs on the null stream, which does not wait for the context stream's kernels.
hipError_t copy_sync(hipStream_t s, void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, s);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(s);
}
int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
#define HIPCHK(expr)                                                                              \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) return fail(DMX_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// Caching device allocator for the large per-graph buffers (run pool, scan order, visibility rows:
// tens of GB at 1000^2).  hipMalloc/hipFree of such blocks costs seconds per graph; repeated
// analyses of same-sized maps reuse them instead.  Blocks >= 64 MiB are kept per device on free and
// handed out again for requests of at most that size and at least 7/8 of it; an allocation that
// fails releases the whole cache and retries.  All users work on one stream per context, so a
// reused block is ordered after every kernel that touched it before.
struct BlockCache {
    static constexpr size_t kMin = 64ull << 20;
    std::mutex m;
    std::multimap<std::pair<int, size_t>, void*> free_blocks;   // (device, bytes) -> block
    std::map<void*, std::pair<int, size_t>> live;                // cached-size blocks handed out
    size_t cached = 0;
    void release_all() {
        for (auto& kv : free_blocks) (void)hipFree(kv.second);
        free_blocks.clear();
        cached = 0;
    }
    // blocks cached on one device: what an allocation failure there can get back
    size_t cached_on(int dev) const {
        size_t b = 0;
        for (auto it = free_blocks.lower_bound({dev, 0}); it != free_blocks.end() && it->first.first == dev; ++it)
            b += it->first.second;
        return b;
    }
};
BlockCache& block_cache() {
    static BlockCache* c = new BlockCache();   // never destroyed: frees at exit would race the runtime
    return *c;
}
// the blocks the cache holds for the current device (added to hipMemGetInfo's free memory: an
// allocation failure releases them)
size_t cached_bytes() {
    BlockCache& c = block_cache();
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(c.m);
    return c.cached_on(dev);
}
hipError_t cached_malloc(void** p, size_t bytes) {
    BlockCache& c = block_cache();
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (bytes >= BlockCache::kMin) {
        bool hit = false;
        {
            std::lock_guard<std::mutex> g(c.m);
            auto it = c.free_blocks.lower_bound({dev, bytes});
            if (it != c.free_blocks.end() && it->first.first == dev && it->first.second - it->first.second / 8 <= bytes) {
                *p = it->second;
                c.cached -= it->first.second;
                c.live[*p] = it->first;
                c.free_blocks.erase(it);
                hit = true;
            }
        }
        // a cached block may have been freed by another context while kernels on its stream still used
        // it: wait for the device before handing it out again (what hipFree would have done)
        if (hit) return hipDeviceSynchronize();
    }
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) {
        std::lock_guard<std::mutex> g(c.m);
        if (c.cached) {
            (void)hipGetLastError();
            c.release_all();
            e = hipMalloc(p, bytes);
        }
    }
    if (e == hipSuccess && bytes >= BlockCache::kMin) {
        std::lock_guard<std::mutex> g(c.m);
        c.live[*p] = {dev, bytes};
    }
    return e;
}
void cached_free(void* p) {
    BlockCache& c = block_cache();
    {
        std::lock_guard<std::mutex> g(c.m);
        auto it = c.live.find(p);
        if (it != c.live.end()) {
            c.free_blocks.insert({it->second, p});
            c.cached += it->second.second;
            c.live.erase(it);
            return;
        }
    }
    (void)hipFree(p);
}

template <typename T> struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    ~DevBuf() { reset(); }
    void reset() {
        if (p) cached_free(p);
        p = nullptr;
        n = 0;
    }
    hipError_t alloc(size_t count) {
        if (count <= n && p) return hipSuccess;
        reset();
        hipError_t e = cached_malloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T));
        if (e == hipSuccess) n = count;
        return e;
    }
};
} // namespace

struct dmx_ctx {
    int device = 0;
    bool tile_disabled = false;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int num_cu = 0;
    double last_mk_s = 0, last_vga_s = 0, last_sd_s = 0;
    long long last_sd_stats[3] = {0, 0, 0};   // expanders popped, cells relaxed, batches (serial: refills)
    long long last_sd_extra[2] = {0, 0};      // batched: improved cells, ambiguous cells
    int last_sd_mode = 0;                     // 0 serial, 1 batched, 2 batched overflow -> serial
    long long phase_cycles[5] = {0, 0, 0, 0, 0};   // tile BFS: level 1, A, B, C, bookkeeping (sum over workgroups)
    DevBuf<int> counters;   // [0] work counter, [1] error word, [2..3] pool cursor (u64)
    DevBuf<unsigned long long> stats; // [0..1] makegraph, [4..6] vga
    long long last_stats[48] = {};
    std::vector<int64_t> last_mk_reruns;   // sources the last makeGraph re-ran (MK_CAPACITY_TAG: capacity)
    // progress / cancel (dmx_ctx_set_progress, dmx_ctx_cancel): host-mapped block polled by the kernels
    DmxCtl* h_ctl = nullptr;
    DmxCtl* d_ctl = nullptr;
    dmx_progress_fn progress = nullptr;
    void* progress_user = nullptr;
    double progress_interval = 0.5;
    hipEvent_t ev_poll = nullptr;
    double last_fill_s[2] = {0, 0};   // GPU fill: blockLines, flood fill
    double sqrt_err = 0.0;            // makeGraph moment square root: measured error bound (mk_sqrt_err)
    long long sqrt_err_nmax = 0;      // ... over 1..sqrt_err_nmax
    long long last_fill_levels = 0;
};

struct dmx_pointmap {
    std::unique_ptr<PointMapHost> host;
    // device copies (per context device; refreshed when the host state changes)
    int uploaded_for = -1;
    uint64_t version = 1, uploaded_version = 0;
    int64_t nnodes = 0;
    std::vector<int32_t> node_cell;
    DevBuf<uint32_t> d_cellw;
    DevBuf<double> d_segs;
    DevBuf<int32_t> d_node_cell;
    DevBuf<int32_t> d_cell_node;
    DevBuf<uint8_t> d_node_flags;
    DevBuf<unsigned long long> d_seed_tiles;
    DevBuf<unsigned long long> d_nonexp_tiles;  // contextfilled cells with odd x or y
};

struct dmx_graph {
    dmx_ctx* ctx = nullptr;
    dmx_pointmap* pm = nullptr;
    // merge links (Point::m_merge): unique pairs (a < b) of x-major cells; device copies built by
    // prepare_merges for the searches that follow them
    std::vector<int32_t> merges;
    bool merges_ready = false;
    DevBuf<int2> d_mpairs;           // [m] (a, b) cells
    DevBuf<int2> d_mamb;             // links with exactly one end context-filled at an odd PixelRef: (that end, the other)
    int nmamb = 0;
    DevBuf<int32_t> d_merge_cell;    // [C] partner cell or -1
    int64_t nnodes = 0, node_begin = 0, node_end = 0;
    int64_t nruns = 0;
    DevBuf<Run> pool;
    DevBuf<int64_t> node_run_start;
    DevBuf<int32_t> node_nruns;
    DevBuf<int32_t> bin_nruns;
    DevBuf<uint16_t> bin_count;
    DevBuf<float> bin_dist;
    DevBuf<float> attrs;
    DevBuf<uint8_t> gridconn;
    // VGA early-exit universe
    DevBuf<unsigned long long> uf_tiles;
    DevBuf<unsigned long long> notuf_tiles;
    int64_t uf_count = -1;
    bool scan_ready = false;   // prepare_uf done (scan order; U_f from the symmetry pass or coverage counting)
    bool scan_released = false;   // the scan order gave its memory to the wide-grid masks (runs read in pool order)
    // bottom-up scan order: runs of each node longest-first, indexed by cell
    DevBuf<Run> scan_pool;
    DevBuf<int64_t> cell_scan_start;
    DevBuf<int32_t> cell_nruns;
    DevBuf<int64_t> scan_start;   // [N] start of each node's runs in scan_pool
    int symmetric = -1;   // -1 unknown, 0 top-down only, 1 bottom-up allowed (with corrections)
    int nspecial = 0;
    std::vector<int32_t> special_nodes;
    DevBuf<int32_t> spec_index, extra_off, extra, missing_off, missing;
    // the symmetry scatter done by makeGraph as it published the runs (sym_fused): consumed and freed by
    // prepare_symmetry
    DevBuf<unsigned long long> sym_prefix, sym_diff, sym_ho;
    bool sym_fused = false;
    // tile-resolved BFS (vga_tile.hip)
    bool tiles_ready = false;
    DevBuf<int64_t> tscan_start;
    DevBuf<int32_t> tnruns;
    DevBuf<Run> heads, cr;
    DevBuf<unsigned long long> tvis;   // tile-visibility rows (empty: not built / too large)
    DevBuf<unsigned long long> ftvis;  // full-visibility rows (every non-seed cell of the tile seen)
    DevBuf<unsigned long long> ttvis;  // tile-to-tile full visibility (AND of ftvis over regular cells)
    DevBuf<unsigned long long> tvsum;  // wide grids: per cell, one bit per non-zero tvis row word
    DevBuf<unsigned long long> tvnz;   // grids up to 256 row words: the same (phase C skips the zero words)
    DevBuf<unsigned long long> pmask;  // partial-tile masks (the cells of each partly seen tile a cell sees)
    DevBuf<int64_t> poff;              // [Ct + 1] start of each cell's masks
    DevBuf<uint16_t> ppre;             // [Ct][tvw] partial tiles of a cell before each row word
    int tvw = 0;
    DevBuf<unsigned long long> regular_tiles;
    // sharded VGA preparation (dmx_graph_set_prep_shard): the node scatters run over [prep_b, prep_e)
    // and the partial buffers are summed across ranks by the caller's all-reduce
    int64_t prep_b = 0, prep_e = -1;
    dmx_allreduce_fn prep_fn = nullptr;
    void* prep_user = nullptr;
    // asymmetric mode (prepare_asym): the drawing the graph's map was made from (dmx_graph_set_drawing), the
    // symmetric reference graph R made from it again, and A, the nodes whose runs differ from R's (plus R's own
    // asymmetric nodes), as a tile bitmap
    std::vector<double> drawing;
    bool has_drawing = false;
    int asym_state = 0;   // 0 not tried, 1 ready, -1 not usable (reason in asym_why)
    std::string asym_why;
    std::unique_ptr<dmx_pointmap> aref_pm;
    std::unique_ptr<dmx_graph> aref;
    DevBuf<unsigned long long> asym_tiles;
    int64_t nasym = 0;
    ~dmx_graph();
};
dmx_graph::~dmx_graph() = default;

namespace {

// A graph made from a point map follows the map's merge links (Point::m_merge of its points).
void inherit_merges(dmx_graph* g) {
    const std::vector<int32_t>& pc = g->pm->host->merge();
    g->merges.clear();
    for (size_t c = 0; c < pc.size(); c++)
        if (pc[c] > (int32_t)c) { g->merges.push_back((int32_t)c); g->merges.push_back(pc[c]); }
    g->merges_ready = false;
}

// Device copies of the merge links for the searches; every linked cell must hold a node (the reference
// calls getNode() on the partner, vgavisualglobal.cpp:116-118).  Links with exactly one end CONTEXTFILLED at
// an odd PixelRef are also listed end-first (d_mamb): where the analysis does not expand that end (a radius,
// visual step depth) a source that finds both ends at one level gets the reference's result only in one pop
// order (merge_order_check, vsd_merge_kernel), and such a source is refused rather than guessed.
int prepare_merges(dmx_graph* g) {
    if (!g || g->merges_ready || g->merges.empty()) return DMX_OK;   // (a NULL graph fails in the caller)
    HIPCHK(hipSetDevice(g->ctx->device));
    const PointMapHost& h = *g->pm->host;
    const int64_t C = h.cells(), m = (int64_t)g->merges.size() / 2;
    const auto& st = h.state();
    const int rows = h.rows();
    auto cf_odd = [&](int32_t c) {
        const int x = c / rows, y = c % rows;
        return (st[c] & CELL_CONTEXTFILLED) && !((x % 2) == 0 && (y % 2) == 0);
    };
    std::vector<int32_t> per_cell((size_t)C, -1);
    std::vector<int2> pairs((size_t)m), amb;
    for (int64_t i = 0; i < m; i++) {
        const int32_t a = g->merges[2 * i], b = g->merges[2 * i + 1];
        if (!(st[a] & CELL_FILLED) || !(st[b] & CELL_FILLED)) return fail(DMX_ERR_ARG, "merge link to a cell without a node");
        per_cell[a] = b;
        per_cell[b] = a;
        pairs[i] = make_int2(a, b);
        if (cf_odd(a) != cf_odd(b)) amb.push_back(cf_odd(a) ? make_int2(a, b) : make_int2(b, a));
    }
    HIPCHK(g->d_mpairs.alloc(m));
    HIPCHK(g->d_merge_cell.alloc(C));
    HIPCHK(hipMemcpyAsync(g->d_mpairs.p, pairs.data(), m * sizeof(int2), hipMemcpyHostToDevice, g->ctx->stream));
    HIPCHK(hipMemcpyAsync(g->d_merge_cell.p, per_cell.data(), C * 4, hipMemcpyHostToDevice, g->ctx->stream));
    g->nmamb = (int)amb.size();
    if (g->nmamb) {
        HIPCHK(g->d_mamb.alloc(amb.size()));
        HIPCHK(hipMemcpyAsync(g->d_mamb.p, amb.data(), amb.size() * sizeof(int2), hipMemcpyHostToDevice, g->ctx->stream));
    }
    HIPCHK(hipStreamSynchronize(g->ctx->stream));
    g->merges_ready = true;
    return DMX_OK;
}

// makeGraph's span certificate (makegraph.hip): every clean cell (FILLED, no occluder piece) gets in its cell
// word, in place of the unused segment offset, its clean distance -- the Chebyshev distance to the nearest cell
// that is not clean or lies outside the grid.  Two raster passes of the 8-neighbour chamfer (Rosenfeld-Pfaltz),
// exact for the Chebyshev metric; the outside enters as each cell's distance to the border.
static void clean_distance(const PointMapHost& h, std::vector<uint32_t>& cellw) {
    const int W = h.cols(), H = h.rows();
    std::vector<uint32_t> d((size_t)W * H);
    for (int x = 0; x < W; x++)
        for (int y = 0; y < H; y++) {
            const size_t c = (size_t)x * H + y;
            const bool clean = (cellw[c] & 0xFFu) == 1u;   // FILLED, 0 pieces
            d[c] = clean ? (uint32_t)std::min(std::min(x + 1, y + 1), std::min(W - x, H - y)) : 0u;
        }
    for (int x = 0; x < W; x++)
        for (int y = 0; y < H; y++) {
            const size_t c = (size_t)x * H + y;
            uint32_t v = d[c];
            if (!v) continue;
            if (y > 0) v = std::min(v, d[c - 1] + 1);
            if (x > 0) {
                const size_t l = c - H;
                v = std::min(v, d[l] + 1);
                if (y > 0) v = std::min(v, d[l - 1] + 1);
                if (y + 1 < H) v = std::min(v, d[l + 1] + 1);
            }
            d[c] = v;
        }
    for (int x = W - 1; x >= 0; x--)
        for (int y = H - 1; y >= 0; y--) {
            const size_t c = (size_t)x * H + y;
            uint32_t v = d[c];
            if (!v) continue;
            if (y + 1 < H) v = std::min(v, d[c + 1] + 1);
            if (x + 1 < W) {
                const size_t r = c + H;
                v = std::min(v, d[r] + 1);
                if (y > 0) v = std::min(v, d[r - 1] + 1);
                if (y + 1 < H) v = std::min(v, d[r + 1] + 1);
            }
            d[c] = v;
        }
    for (size_t c = 0; c < d.size(); c++)
        if ((cellw[c] & 0xFFu) == 1u) cellw[c] = (std::min(d[c], CELL_DIST_MAX) << 8) | 1u;
}

int upload_pointmap(dmx_ctx* ctx, dmx_pointmap* pm) {
    PointMapHost& h = *pm->host;
    if (!h.lines_blocked()) h.block_lines();
    if (pm->uploaded_version == pm->version && pm->uploaded_for == ctx->device) return DMX_OK;
    if (pm->uploaded_for >= 0 && pm->uploaded_for != ctx->device) {
        // another device's copies: release them (DevBuf::alloc would otherwise reuse the pointers)
        pm->d_cellw.reset(); pm->d_segs.reset(); pm->d_node_cell.reset(); pm->d_cell_node.reset();
        pm->d_node_flags.reset(); pm->d_seed_tiles.reset(); pm->d_nonexp_tiles.reset();
        pm->uploaded_for = -1;
    }
    const int64_t C = h.cells();
    std::vector<uint32_t> cellw((size_t)C);
    const auto& st = h.state();
    const auto& off = h.seg_off();
    pm->node_cell.clear();
    std::vector<int32_t> cell_node((size_t)C, -1);
    std::vector<uint8_t> flags;
    for (int64_t c = 0; c < C; c++) {
        const int32_t n = off[c + 1] - off[c];
        if (n > 127) return fail(DMX_ERR_UNSUPPORTED, "more than 127 occluder pieces in one grid cell");
        if ((int64_t)off[c] >= (1 << 24)) return fail(DMX_ERR_UNSUPPORTED, "more than 16M occluder pieces");
        const bool filled = st[c] & CELL_FILLED;
        cellw[c] = pack_cell(filled, (uint32_t)n, (uint32_t)off[c]);
        if (filled) {
            cell_node[c] = (int32_t)pm->node_cell.size();
            pm->node_cell.push_back((int32_t)c);
            flags.push_back((st[c] & CELL_CONTEXTFILLED) ? 1 : 0);
        }
    }
    pm->nnodes = (int64_t)pm->node_cell.size();
    clean_distance(h, cellw);
    // seed bitmap for the BFS: 1 = not a filled cell (or padding), 8x8 tiles
    const int tw = (h.cols() + 7) / 8, th = (h.rows() + 7) / 8;
    std::vector<unsigned long long> seed((size_t)tw * th, ~0ull), nonexp((size_t)tw * th, 0ull);
    for (int x = 0; x < h.cols(); x++)
        for (int y = 0; y < h.rows(); y++) {
            const int32_t sv = st[h.index(x, y)];
            const unsigned long long bit = 1ull << ((y & 7) * 8 + (x & 7));
            if (sv & CELL_FILLED) seed[(size_t)(y >> 3) * tw + (x >> 3)] &= ~bit;
            if ((sv & CELL_CONTEXTFILLED) && !((x % 2) == 0 && (y % 2) == 0)) nonexp[(size_t)(y >> 3) * tw + (x >> 3)] |= bit;
        }
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(pm->d_cellw.alloc(C));
    HIPCHK(pm->d_segs.alloc(std::max<size_t>(h.segs().size(), 4)));
    HIPCHK(pm->d_node_cell.alloc(std::max<int64_t>(pm->nnodes, 1)));
    HIPCHK(pm->d_cell_node.alloc(C));
    HIPCHK(pm->d_node_flags.alloc(std::max<int64_t>(pm->nnodes, 1)));
    HIPCHK(pm->d_seed_tiles.alloc(seed.size()));
    HIPCHK(pm->d_nonexp_tiles.alloc(nonexp.size()));
    HIPCHK(hipMemcpyAsync(pm->d_nonexp_tiles.p, nonexp.data(), nonexp.size() * 8, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(pm->d_cellw.p, cellw.data(), C * 4, hipMemcpyHostToDevice, ctx->stream));
    if (!h.segs().empty())
        HIPCHK(hipMemcpyAsync(pm->d_segs.p, h.segs().data(), h.segs().size() * 8, hipMemcpyHostToDevice, ctx->stream));
    if (pm->nnodes) {
        HIPCHK(hipMemcpyAsync(pm->d_node_cell.p, pm->node_cell.data(), pm->nnodes * 4, hipMemcpyHostToDevice, ctx->stream));
        HIPCHK(hipMemcpyAsync(pm->d_node_flags.p, flags.data(), pm->nnodes, hipMemcpyHostToDevice, ctx->stream));
    }
    HIPCHK(hipMemcpyAsync(pm->d_cell_node.p, cell_node.data(), C * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(pm->d_seed_tiles.p, seed.data(), seed.size() * 8, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    pm->uploaded_version = pm->version;
    pm->uploaded_for = ctx->device;
    return DMX_OK;
}

__global__ void node_nruns_kernel(const int32_t* bin_nruns, int64_t n, int32_t* out) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    int s = 0;
    for (int b = 0; b < 32; b++) s += bin_nruns[k * 32 + b];
    out[k] = s;
}

// copy each node's runs to a contiguous node-ordered destination
__global__ void gather_runs_kernel(const Run* pool, const int64_t* start, const int32_t* nruns, const int64_t* dst_off,
                                   int64_t n, Run* dst) {
    int64_t k = blockIdx.x;
    if (k >= n) return;
    const int64_t s = start[k], d = dst_off[k];
    for (int i = threadIdx.x; i < nruns[k]; i += blockDim.x) dst[d + i] = pool[s + i];
}

// Merge links as unique pairs (a < b): both directions of a pair may be listed (PointMap::write stores
// m_merge on both points), every cell belongs to at most one pair (PointMap::mergePixels,
// pointdata.cpp:1653-1680, unlinks a cell's previous partner).  per_cell[c] = partner or -1.
int normalize_merges(int64_t C, const int32_t* pairs, int64_t n, std::vector<int32_t>& per_cell,
                     std::vector<int32_t>& uniq, bool both_ways = false) {
    per_cell.assign(n ? (size_t)C : 0, -1);
    uniq.clear();
    std::vector<int32_t> from;   // both_ways: the partner each cell's own entry names
    if (both_ways && n) from.assign((size_t)C, -1);
    for (int64_t i = 0; i < n; i++) {
        const int32_t a = pairs[2 * i], b = pairs[2 * i + 1];
        if (a < 0 || b < 0 || a >= C || b >= C || a == b) return fail(DMX_ERR_ARG, "merge link outside the grid");
        if ((per_cell[a] >= 0 && per_cell[a] != b) || (per_cell[b] >= 0 && per_cell[b] != a))
            return fail(DMX_ERR_ARG, "a cell with two merge links");
        if (per_cell[a] < 0) { uniq.push_back(std::min(a, b)); uniq.push_back(std::max(a, b)); }
        per_cell[a] = b;
        per_cell[b] = a;
        if (both_ways) from[a] = b;
    }
    // a saved map stores a link on both points (PointMap::mergePixels sets m_merge on each, pointdata.cpp:
    // 1653-1680), and the searches follow the merge pixel of the point they pop (vgavisualglobal.cpp:113): a
    // link stored on one end only would be followed one way by the reference -- refused, not made two-way
    if (both_ways)
        for (size_t i = 0; i < uniq.size(); i += 2)
            if (from[uniq[i]] != uniq[i + 1] || from[uniq[i + 1]] != uniq[i])
                return fail(DMX_ERR_ARG, "a merge link stored on one of its points only (damaged map)");
    return DMX_OK;
}

size_t makegraph_lds(int gcap, int bcap, int D) {
    size_t b = 0;
    b += 16 * (size_t)gcap * 2 + 16 * (size_t)bcap; // gaps, gaps2, blocks
    b += 4 * 32 * 3 + 4 * 32;                        // binc, bfar, bnr, misc
    b += 16 * (size_t)bcap;                          // bsorted
    b += 4 * (size_t)gcap + 8 * (size_t)gcap + 4 * (size_t)bcap + 4 * ((size_t)gcap + 4);
    b += 4 * (size_t)std::min(D + 4, MK_OPEN_LDS);   // open-run state of the near rows (makegraph.hip)
    return (b + 15) & ~(size_t)15;
}

} // namespace

// Diagnostics (DMX_ABORT_BACKTRACE=1): SIGABRT / SIGSEGV print the native stack (frames as
// module+offset, resolved offline with addr2line against the same build) before the previously
// installed handler (Python's faulthandler) runs.
namespace {
struct sigaction g_prev_abrt, g_prev_segv;
void dmx_crash_handler(int sig, siginfo_t* info, void* uc) {
    void* frames[64];
    const int n = backtrace(frames, 64);
    const char hdr[] = "[dmx] native backtrace:\n";
    (void)!write(2, hdr, sizeof(hdr) - 1);
    backtrace_symbols_fd(frames, n, 2);
    struct sigaction* prev = sig == SIGABRT ? &g_prev_abrt : &g_prev_segv;
    sigaction(sig, prev, nullptr);
    if (prev->sa_flags & SA_SIGINFO) {
        if (prev->sa_sigaction) prev->sa_sigaction(sig, info, uc);
    } else if (prev->sa_handler != SIG_DFL && prev->sa_handler != SIG_IGN) {
        prev->sa_handler(sig);
    }
    raise(sig);
}
void install_crash_handler() {
    static bool done = false;
    const char* e = getenv("DMX_ABORT_BACKTRACE");
    if (done || !e || strcmp(e, "1") != 0) return;
    done = true;
    void* warm[2];
    backtrace(warm, 2);   // loads the unwinder now: the handler must not allocate (the heap may be broken)
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = dmx_crash_handler;
    sa.sa_flags = SA_SIGINFO;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGABRT, &sa, &g_prev_abrt);
    sigaction(SIGSEGV, &sa, &g_prev_segv);
}
} // namespace

extern "C" {

int dmx_abi_version(void) { return DMX_ABI_VERSION; }
const char* dmx_last_error(void) { return g_err.c_str(); }

int dmx_ctx_create(int device, dmx_ctx** out) {
    if (!out) return fail(DMX_ERR_ARG, "out is NULL");
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(DMX_ERR_ARG, "device ordinal out of range");
    HIPCHK(hipSetDevice(device));
    install_crash_handler();
    auto* c = new dmx_ctx();
    c->device = device;
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    c->num_cu = prop.multiProcessorCount;
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHK(hipEventCreate(&c->ev0));
    HIPCHK(hipEventCreate(&c->ev1));
    HIPCHK(c->counters.alloc(16));
    HIPCHK(c->stats.alloc(32));
    HIPCHK(hipEventCreateWithFlags(&c->ev_poll, hipEventDisableTiming));
    HIPCHK(hipHostMalloc((void**)&c->h_ctl, sizeof(DmxCtl), hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(c->h_ctl, 0, sizeof(DmxCtl));
    HIPCHK(hipHostGetDevicePointer((void**)&c->d_ctl, c->h_ctl, 0));
    *out = c;
    return DMX_OK;
}

int dmx_ctx_set_progress(dmx_ctx* ctx, dmx_progress_fn fn, void* user, double interval_s) {
    if (!ctx || interval_s != interval_s) return fail(DMX_ERR_ARG, "bad arguments");   // NaN only: <= 0 means 0.5 s
    ctx->progress = fn;
    ctx->progress_user = user;
    ctx->progress_interval = interval_s > 0.0 ? interval_s : 0.5;
    return DMX_OK;
}

int dmx_ctx_cancel(dmx_ctx* ctx) {
    if (!ctx || !ctx->h_ctl) return fail(DMX_ERR_ARG, "bad context");
    __atomic_store_n(&ctx->h_ctl->cancel, 1, __ATOMIC_SEQ_CST);
    return DMX_OK;
}

// Wait for the work queued on the context stream.  With a progress callback, poll it every interval
// while the kernel runs: done = (work items taken, published by the kernel) x unit; a non-zero return
// from the callback requests cancellation, as dmx_ctx_cancel does.
static hipError_t wait_progress(dmx_ctx* ctx, int32_t phase, int64_t total, int64_t unit) {
    if (!ctx->progress) return hipStreamSynchronize(ctx->stream);
    hipError_t e = hipEventRecord(ctx->ev_poll, ctx->stream);
    if (e != hipSuccess) return e;
    double next = now_s() + ctx->progress_interval;
    for (;;) {
        e = hipEventQuery(ctx->ev_poll);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) return e;
        if (now_s() >= next) {
            const int64_t done = std::min<int64_t>(total, (int64_t)__atomic_load_n(&ctx->h_ctl->progress,
                                                                                  __ATOMIC_RELAXED) * unit);
            if (ctx->progress(ctx->progress_user, phase, done, total)) dmx_ctx_cancel(ctx);
            next = now_s() + ctx->progress_interval;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(500));
    }
    if (!__atomic_load_n(&ctx->h_ctl->cancel, __ATOMIC_SEQ_CST) && ctx->progress(ctx->progress_user, phase, total, total))
        dmx_ctx_cancel(ctx);
    return hipSuccess;
}

// A raised cancel flag ends the running operation with DMX_ERR_CANCELLED and is consumed by it.
static bool take_cancel(dmx_ctx* ctx) {
    if (!__atomic_load_n(&ctx->h_ctl->cancel, __ATOMIC_SEQ_CST)) return false;
    __atomic_store_n(&ctx->h_ctl->cancel, 0, __ATOMIC_SEQ_CST);
    return true;
}
// a graph lives on the device of the context that built it
#define SAME_DEVICE(ctx, g)                                                                          \
    do {                                                                                             \
        if ((ctx) && (g) && (g)->ctx && (g)->ctx->device != (ctx)->device)                           \
            return fail(DMX_ERR_ARG, "graph was built on another device than the context's");        \
    } while (0)
#define CANCEL_POINT(ctx)                                                        \
    do {                                                                         \
        if (take_cancel(ctx)) return fail(DMX_ERR_CANCELLED, "operation cancelled"); \
    } while (0)

int dmx_release_cached_memory(void) {
    BlockCache& c = block_cache();
    std::lock_guard<std::mutex> g(c.m);
    c.release_all();
    return DMX_OK;
}

int dmx_ctx_free(dmx_ctx* c) {
    if (!c) return DMX_OK;
    (void)hipSetDevice(c->device);
    c->counters.reset();
    c->stats.reset();
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->ev_poll) (void)hipEventDestroy(c->ev_poll);
    if (c->h_ctl) (void)hipHostFree(c->h_ctl);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return DMX_OK;
}

int dmx_ctx_last_stats(dmx_ctx* c, int64_t* out, int n) {
    if (!c || !out) return fail(DMX_ERR_ARG, "bad arguments");
    for (int i = 0; i < n && i < 48; i++) out[i] = c->last_stats[i];
    return DMX_OK;
}

int dmx_ctx_last_timing(dmx_ctx* c, double* mk, double* vga) {
    if (!c) return fail(DMX_ERR_ARG, "ctx is NULL");
    if (mk) *mk = c->last_mk_s;
    if (vga) *vga = c->last_vga_s;
    return DMX_OK;
}

#include "api/pointmap.hip"
#include "api/makegraph.hip"
#include "api/shard.hip"
#include "api/vga_global.hip"
#include "api/vga_other.hip"
#include "api/stepdepth.hip"
#include "api/chunk.hip"
#include "api/graphfile.hip"

} // extern "C"
