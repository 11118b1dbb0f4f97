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

int dmx_pointmap_create(const double* region, double spacing, const double* lines, int64_t nlines, dmx_pointmap** out) {
    if (!region || !out || (nlines > 0 && !lines) || nlines < 0) return fail(DMX_ERR_ARG, "bad arguments");
    if (!(spacing > 0)) return fail(DMX_ERR_ARG, "spacing must be > 0");
    Rect r{region[0], region[1], region[2], region[3]};
    auto* pm = new dmx_pointmap();
    pm->host.reset(new PointMapHost(r, spacing, lines, nlines));
    if (pm->host->cols() > 16000 || pm->host->rows() > 16000) {
        delete pm;
        return fail(DMX_ERR_UNSUPPORTED, "grid larger than 16000 cells per side");
    }
    *out = pm;
    return DMX_OK;
}

int dmx_pointmap_free(dmx_pointmap* pm) {
    delete pm;
    return DMX_OK;
}

int dmx_pointmap_make_points(dmx_pointmap* pm, double x, double y, int fill_type, int* made) {
    if (!pm) return fail(DMX_ERR_ARG, "pointmap is NULL");
    if (made) *made = 0;
    if (PointMapHost::fill_state_of(fill_type) < 0) return fail(DMX_ERR_ARG, "fill_type must be 0, 1 or 2");
    int r = pm->host->fill(x, y, fill_type);
    pm->version++;
    if (made) *made = (r == 0);
    if (r == 1) return fail(DMX_ERR_OUTSIDE, "Point outside of target region");
    if (r == 3)
        return fail(DMX_ERR_UNSUPPORTED, "an AUGMENT fill from this seed never ends in the reference (expand re-queues "
                                         "augmented cells, pointdata.cpp:489)");
    return DMX_OK;
}

int dmx_pointmap_fill(dmx_pointmap* pm, double x, double y, int* made) {
    return dmx_pointmap_make_points(pm, x, y, 0, made);
}

namespace {
// scratch for scan_excl: per level, the tile sums and the tile offsets (+ total)
int64_t scan_scratch_size(int64_t n) {
    int64_t s = 1;
    for (;;) {
        const int64_t t = (n + SCAN_TILE - 1) / SCAN_TILE;
        s += 2 * t + 1;
        if (t <= 1) break;
        n = t;
    }
    return s;
}
// out[0..n) = exclusive prefix of in, out[n] = total; out must not alias in.
void scan_excl(hipStream_t st, const int64_t* in, int64_t n, int64_t* out, int64_t* scratch) {
    if (n <= 0) {
        (void)hipMemsetAsync(out, 0, sizeof(int64_t), st);
        return;
    }
    const int64_t t = (n + SCAN_TILE - 1) / SCAN_TILE;
    int64_t* tsum = scratch;
    int64_t* toff = scratch + t;
    hipLaunchKernelGGL(scan_tile_kernel, dim3((unsigned)t), dim3(SCAN_THREADS), 0, st, in, n, out, tsum);
    if (t == 1) {
        hipLaunchKernelGGL(scan_total_kernel, dim3(1), dim3(1), 0, st, out, n, (const int64_t*)tsum);
        return;
    }
    scan_excl(st, tsum, t, toff, scratch + 2 * t + 1);
    hipLaunchKernelGGL(scan_add_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out, n, (const int64_t*)toff);
    hipLaunchKernelGGL(scan_total_kernel, dim3(1), dim3(1), 0, st, out, n, (const int64_t*)(toff + t));
}
unsigned fill_blocks(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + FILL_THREADS - 1) / FILL_THREADS); }
} // namespace

// PointMap::makePoints on the GPU (kernels/fill.hip): blockLines on the first fill, then the ordered
// level-synchronous flood fill.  The host model stays the owner of the results (cell states,
// cropped pieces), so makeGraph and the .graph writer see exactly what the host fill would leave.
int dmx_pointmap_fill_device(dmx_ctx* ctx, dmx_pointmap* pm, double x, double y, int* made) {
    return dmx_pointmap_make_points_device(ctx, pm, x, y, 0, made);
}

int dmx_pointmap_make_points_device(dmx_ctx* ctx, dmx_pointmap* pm, double x, double y, int fill_type, int* made) {
    if (!ctx || !pm) return fail(DMX_ERR_ARG, "bad arguments");
    PointMapHost& h = *pm->host;
    if (made) *made = 0;
    const int32_t fill_state = PointMapHost::fill_state_of(fill_type);
    if (fill_state < 0) return fail(DMX_ERR_ARG, "fill_type must be 0, 1 or 2");
    // AUGMENT changes the seed cell alone or never ends (PointMapHost::fill): nothing to flood
    if (fill_state == CELL_AUGMENTED) return dmx_pointmap_make_points(pm, x, y, fill_type, made);
    int sx = 0, sy = 0;
    const int r = h.fill_seed(x, y, &sx, &sy);
    if (r == 1) return fail(DMX_ERR_OUTSIDE, "Point outside of target region");
    if (r) return DMX_OK;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const double t0 = now_s();
    const int64_t C = h.cells();
    FillGrid G;
    G.cols = h.cols();
    G.rows = h.rows();
    G.spacing = h.spacing();
    G.blx = h.bottom_left().x;
    G.bly = h.bottom_left().y;
    G.region = h.grid_region();
    DevBuf<int32_t> d_state, d_segoff;
    DevBuf<double> d_segs;
    DevBuf<int64_t> cnt, off, scratch;
    HIPCHK(d_state.alloc(C));
    HIPCHK(d_segoff.alloc(C + 1));
    HIPCHK(cnt.alloc(C + 1));
    HIPCHK(off.alloc(C + 1));
    HIPCHK(scratch.alloc(scan_scratch_size(C + 1)));
    HIPCHK(hipMemcpyAsync(d_state.p, h.state().data(), C * sizeof(int32_t), hipMemcpyHostToDevice, st));
    int64_t npieces = 0;
    if (!h.lines_blocked()) {
        // blockLines: count / scan / emit per line, place / sort / crop per cell
        const std::vector<double>& draw = h.drawing();
        const int64_t L = (int64_t)draw.size() / 4;
        DevBuf<double> d_draw;
        DevBuf<int64_t> line_off, cursor;
        DevBuf<int32_t> em_cell, cell_lines;
        HIPCHK(d_draw.alloc(std::max<int64_t>(4 * L, 1)));
        HIPCHK(line_off.alloc(L + 1));
        if (L) HIPCHK(hipMemcpyAsync(d_draw.p, draw.data(), 4 * L * sizeof(double), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemsetAsync(cnt.p, 0, (C + 1) * sizeof(int64_t), st));
        DevBuf<int64_t> lcnt, lscratch;
        HIPCHK(lcnt.alloc(std::max<int64_t>(L, 1)));
        HIPCHK(lscratch.alloc(scan_scratch_size(L)));
        if (L) hipLaunchKernelGGL(rast_count_kernel, dim3(fill_blocks(L)), dim3(FILL_THREADS), 0, st, G, (const double*)d_draw.p, L, lcnt.p);
        scan_excl(st, lcnt.p, L, line_off.p, lscratch.p);
        int64_t E = 0;
        HIPCHK(copy_sync(st, &E, line_off.p + L, sizeof(int64_t), hipMemcpyDeviceToHost));
        HIPCHK(em_cell.alloc(std::max<int64_t>(E, 1)));
        HIPCHK(cell_lines.alloc(std::max<int64_t>(E, 1)));
        HIPCHK(cursor.alloc(C + 1));
        HIPCHK(hipMemsetAsync(cursor.p, 0, C * sizeof(int64_t), st));
        if (L) hipLaunchKernelGGL(rast_emit_kernel, dim3(fill_blocks(L)), dim3(FILL_THREADS), 0, st, G, (const double*)d_draw.p, L,
                                  (const int64_t*)line_off.p, em_cell.p, cnt.p);
        scan_excl(st, cnt.p, C, off.p, scratch.p);   // off = per-cell line lists
        if (E) hipLaunchKernelGGL(rast_place_kernel, dim3(fill_blocks(E)), dim3(FILL_THREADS), 0, st, (const int64_t*)line_off.p, L,
                                  (const int32_t*)em_cell.p, E, (const int64_t*)off.p, cursor.p, cell_lines.p);
        // cnt is reused for the surviving pieces per cell; cursor (int64) holds their offsets
        hipLaunchKernelGGL(rast_crop_count_kernel, dim3(fill_blocks(C)), dim3(FILL_THREADS), 0, st, G, (const double*)d_draw.p, C,
                           (const int64_t*)off.p, cell_lines.p, d_state.p, cnt.p);
        scan_excl(st, cnt.p, C, cursor.p, scratch.p);
        HIPCHK(copy_sync(st, &npieces, cursor.p + C, sizeof(int64_t), hipMemcpyDeviceToHost));
        if (npieces >= (int64_t)INT32_MAX / 4) return fail(DMX_ERR_UNSUPPORTED, "too many occluder pieces");
        HIPCHK(d_segs.alloc(std::max<int64_t>(4 * npieces, 1)));
        hipLaunchKernelGGL(rast_crop_write_kernel, dim3(fill_blocks(C)), dim3(FILL_THREADS), 0, st, G, (const double*)d_draw.p, C,
                           (const int64_t*)off.p, (const int32_t*)cell_lines.p, (const int64_t*)cursor.p, d_segs.p);
        std::vector<int64_t> off64((size_t)C + 1);
        std::vector<int32_t> seg_off((size_t)C + 1);
        std::vector<double> segs((size_t)(4 * npieces));
        HIPCHK(hipMemcpyAsync(off64.data(), cursor.p, (C + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, st));
        if (npieces) HIPCHK(hipMemcpyAsync(segs.data(), d_segs.p, 4 * npieces * sizeof(double), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        for (int64_t c = 0; c <= C; c++) seg_off[c] = (int32_t)off64[c];
        HIPCHK(hipMemcpyAsync(d_segoff.p, seg_off.data(), (C + 1) * sizeof(int32_t), hipMemcpyHostToDevice, st));
        h.adopt_blocked(std::move(seg_off), std::move(segs));
        VLOG("fill: blockLines on the GPU (%lld lines, %lld cell touches, %lld pieces) %.3f s\n", (long long)L, (long long)E,
             (long long)npieces, now_s() - t0);
    } else {
        npieces = (int64_t)h.segs().size() / 4;
        HIPCHK(d_segs.alloc(std::max<int64_t>(4 * npieces, 1)));
        HIPCHK(hipMemcpyAsync(d_segoff.p, h.seg_off().data(), (C + 1) * sizeof(int32_t), hipMemcpyHostToDevice, st));
        if (npieces) HIPCHK(hipMemcpyAsync(d_segs.p, h.segs().data(), 4 * npieces * sizeof(double), hipMemcpyHostToDevice, st));
    }
    // the ordered flood fill, one level per round
    const double t1 = now_s();
    DevBuf<int32_t> layer[2];
    DevBuf<uint32_t> owner;
    DevBuf<uint8_t> blocked, children;
    HIPCHK(layer[0].alloc(C));
    HIPCHK(layer[1].alloc(C));
    HIPCHK(owner.alloc(C));
    HIPCHK(blocked.alloc(C));
    HIPCHK(children.alloc(C));
    HIPCHK(hipMemsetAsync(owner.p, 0xFF, C * sizeof(uint32_t), st));
    const int64_t c0 = h.index(sx, sy);
    G.fill_state = fill_state;
    const int32_t seed_state = fill_state | (h.state()[c0] & CELL_BLOCKED);
    const int32_t seed_cell = (int32_t)c0;
    HIPCHK(hipMemcpyAsync(d_state.p + c0, &seed_state, sizeof(int32_t), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(layer[0].p, &seed_cell, sizeof(int32_t), hipMemcpyHostToDevice, st));
    int64_t n = 1, levels = 0;
    int cur = 0;
    DevBuf<long long> io;
    HIPCHK(io.alloc(3));
    const bool wg_on = !getenv("DMX_FILL_GRID");   // test hook: every level grid-wide
    while (n > 0) {
        if (wg_on && n <= FILL_WG_CAP) {
            // small layers: one workgroup runs levels until the fill ends or a layer outgrows the cap
            long long h_io[3] = {(long long)n, (long long)cur, 0};
            HIPCHK(hipMemcpyAsync(io.p, h_io, sizeof(h_io), hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(fill_levels_wg_kernel, dim3(1), dim3(FILL_WG_THREADS), 0, st, G, (const int32_t*)d_segoff.p,
                               (const double*)d_segs.p, d_state.p, layer[0].p, layer[1].p, owner.p, io.p);
            HIPCHK(hipGetLastError());
            HIPCHK(copy_sync(st, h_io, io.p, sizeof(h_io), hipMemcpyDeviceToHost));
            n = h_io[0];
            cur = (int)h_io[1];
            levels += h_io[2];
            if (n == 0) break;
        }
        hipLaunchKernelGGL(fill_claim_kernel, dim3(fill_blocks(n)), dim3(FILL_THREADS), 0, st, G, (const int32_t*)d_segoff.p,
                           (const double*)d_segs.p, (const int32_t*)d_state.p, (const int32_t*)layer[cur].p, n, owner.p, blocked.p);
        hipLaunchKernelGGL(fill_resolve_kernel, dim3(fill_blocks(n)), dim3(FILL_THREADS), 0, st, G, d_state.p,
                           (const int32_t*)layer[cur].p, n, (const uint32_t*)owner.p, (const uint8_t*)blocked.p, children.p, cnt.p);
        scan_excl(st, cnt.p, n, off.p, scratch.p);
        int64_t n_next = 0;
        HIPCHK(copy_sync(st, &n_next, off.p + n, sizeof(int64_t), hipMemcpyDeviceToHost));
        if (n_next)
            hipLaunchKernelGGL(fill_push_kernel, dim3(fill_blocks(n)), dim3(FILL_THREADS), 0, st, G, d_state.p,
                               (const int32_t*)layer[cur].p, n, (const uint8_t*)children.p, (const int64_t*)off.p, n_next,
                               layer[cur ^ 1].p);
        HIPCHK(hipGetLastError());
        cur ^= 1;
        n = n_next;
        levels++;
    }
    std::vector<int32_t> state((size_t)C);
    HIPCHK(copy_sync(st, state.data(), d_state.p, C * sizeof(int32_t), hipMemcpyDeviceToHost));
    h.adopt_state(std::move(state));
    pm->version++;
    ctx->last_fill_s[0] = t1 - t0;
    ctx->last_fill_s[1] = now_s() - t1;
    ctx->last_fill_levels = levels;
    VLOG("fill: flood fill on the GPU, %lld levels, %lld filled, %.3f s\n", (long long)levels, (long long)h.filled_count(),
         now_s() - t1);
    if (made) *made = 1;
    return DMX_OK;
}

int dmx_ctx_last_fill(dmx_ctx* ctx, double* block_s, double* fill_s, int64_t* levels) {
    if (!ctx) return fail(DMX_ERR_ARG, "ctx is NULL");
    if (block_s) *block_s = ctx->last_fill_s[0];
    if (fill_s) *fill_s = ctx->last_fill_s[1];
    if (levels) *levels = ctx->last_fill_levels;
    return DMX_OK;
}

int dmx_pointmap_info(const dmx_pointmap* pm, int32_t* cols, int32_t* rows, double* bx, double* by, int64_t* filled) {
    if (!pm) return fail(DMX_ERR_ARG, "pointmap is NULL");
    if (cols) *cols = pm->host->cols();
    if (rows) *rows = pm->host->rows();
    if (bx) *bx = pm->host->bottom_left().x;
    if (by) *by = pm->host->bottom_left().y;
    if (filled) *filled = pm->host->filled_count();
    return DMX_OK;
}

int dmx_pointmap_state(const dmx_pointmap* pm, int32_t* out) {
    if (!pm || !out) return fail(DMX_ERR_ARG, "bad arguments");
    std::memcpy(out, pm->host->state().data(), pm->host->state().size() * 4);
    return DMX_OK;
}

int dmx_pointmap_cell_lines(dmx_pointmap* pm, int32_t* counts, double* pieces, int64_t* total) {
    if (!pm) return fail(DMX_ERR_ARG, "pointmap is NULL");
    pm->host->block_lines();
    const auto& off = pm->host->seg_off();
    const auto& segs = pm->host->segs();
    if (total) *total = (int64_t)segs.size() / 4;
    if (counts)
        for (size_t c = 0; c + 1 < off.size(); c++) counts[c] = off[c + 1] - off[c];
    if (pieces && !segs.empty()) std::memcpy(pieces, segs.data(), segs.size() * 8);
    return DMX_OK;
}

// makeGraph kernel variants (makegraph.hip).  VGPR budget: 5 waves per SIMD.  The kernel is latency-bound
// (one wave walks one source's sieve depth by depth), so waves beat registers: at 1000^2, 3 waves/SIMD
// 6.9 s, 4: 5.4 s, 5: 4.9 s (96 VGPRs, some cold spills), 6: 5.4 s.  fixed: the first pass (LDS
// capacities, certified moment sums and the maxdist test compiled in); count: the cost-sample counters.
typedef void (*mk_kernel_t)(const MakeGraphParams*);
// waves per SIMD the makeGraph register allocation targets (A/B builds: -DDMX_MK_WPE=n).  Measured round 4
// (profiles/r4_makegraph_wpe_ab.jsonl, configs[2] / configs[4]): 5 -> 4.62 / 10.65 s, 6 -> 5.20 / 11.99 s,
// 8 -> 9.10 / 19.31 s: fewer registers spill more than the extra waves hide
#ifndef DMX_MK_WPE
#define DMX_MK_WPE 5
#endif
#define MKK(PROF, FIXED, COUNT, MAXD, FAR) makegraph_kernel<DMX_MK_WPE, PROF, FIXED, COUNT, MAXD, FAR>
static mk_kernel_t mk_kernel(bool fixed, bool count, bool maxd, bool far) {
    if (count) {       // the cost sample of dmx_makegraph_balance: always counts (its bounds depend on it)
        if (!fixed || maxd) return MKK(false, false, true, false, false);
        return far ? MKK(false, true, true, false, true) : MKK(false, true, true, false, false);
    }
    if (verbose()) {   // per-phase clocks (maxdist runs take the generic kernel)
        if (!fixed || maxd) return MKK(true, false, false, false, false);
        return far ? MKK(true, true, false, false, true) : MKK(true, true, false, false, false);
    }
    if (!fixed) return MKK(false, false, false, false, false);
    if (maxd) return far ? MKK(false, true, false, true, true) : MKK(false, true, false, true, false);
    return far ? MKK(false, true, false, false, true) : MKK(false, true, false, false, false);
}
#undef MKK

// The largest relative error of makeGraph's moment square root (MK_SQRT) over the integers 1..nmax, measured
// exhaustively on the device (once per context and range): the certificate of the moment sums rests on it.
static int mk_sqrt_err(dmx_ctx* ctx, long long nmax, double* err) {
    if (ctx->sqrt_err_nmax < nmax) {
        DevBuf<unsigned long long> e;
        HIPCHK(e.alloc(1));
        HIPCHK(hipMemsetAsync(e.p, 0, 8, ctx->stream));
        hipLaunchKernelGGL(sqrt_err_kernel, dim3((unsigned)std::min<long long>((nmax + 255) / 256, 4096)), dim3(256), 0,
                           ctx->stream, nmax, e.p);
        HIPCHK(hipGetLastError());
        unsigned long long bits = 0;
        HIPCHK(copy_sync(ctx->stream, &bits, e.p, 8, hipMemcpyDeviceToHost));
        double v;
        std::memcpy(&v, &bits, 8);
        // a device square root worse than 2^-30: no source can pass the moment certificate, so every source runs the
        // serial chains (which do not use it) from the first pass (makegraph_impl)
        if (!(v >= 0.0 && v < 0x1p-30)) {
            VLOG("makegraph: square-root error %.3g over 1..%lld: certified moment sums off\n", v, nmax);
            v = INFINITY;
        }
        ctx->sqrt_err = v;
        ctx->sqrt_err_nmax = nmax;
        VLOG("makegraph: square-root error bound %.3g over 1..%lld\n", v, nmax);
    }
    *err = ctx->sqrt_err;
    return DMX_OK;
}

// makeGraph over [node_begin, node_end), or only over the listed nodes of that range (`only`: the cost
// sample of dmx_makegraph_balance; the graph's other nodes stay unset).  d_work (optional, [n][2]) receives
// each published source's sieve depth steps and candidate chunks.
static int makegraph_impl(dmx_ctx* ctx, dmx_pointmap* pm, double maxdist, int boundary, int64_t node_begin,
                          int64_t node_end, const std::vector<int64_t>* only, uint32_t* d_work, dmx_graph** out) {
    if (!ctx || !pm || !out) return fail(DMX_ERR_ARG, "bad arguments");
    HIPCHK(hipSetDevice(ctx->device));
    const double t_start = now_s();
    PointMapHost& h = *pm->host;
    if (!h.lines_blocked()) h.block_lines();
    if (boundary) { h.keep_edges_only(); pm->version++; }
    int rc = upload_pointmap(ctx, pm);
    if (rc) return rc;
    VLOG("makegraph: host prep + upload %.3f s\n", now_s() - t_start);
    const int64_t N = pm->nnodes;
    if (node_end < 0 || node_end > N) node_end = N;
    if (node_begin < 0 || node_begin > node_end) return fail(DMX_ERR_ARG, "bad node range");
    const int64_t n = node_end - node_begin;
    std::unique_ptr<dmx_graph> g(new dmx_graph());
    g->ctx = ctx;
    g->pm = pm;
    g->nnodes = N;
    g->node_begin = node_begin;
    g->node_end = node_end;
    inherit_merges(g.get());
    const int D = std::max(h.cols(), h.rows());
    HIPCHK(g->node_run_start.alloc(std::max<int64_t>(n, 1)));
    HIPCHK(g->node_nruns.alloc(std::max<int64_t>(n, 1)));
    HIPCHK(g->bin_nruns.alloc(std::max<int64_t>(n, 1) * 32));
    HIPCHK(g->bin_count.alloc(std::max<int64_t>(n, 1) * 32));
    HIPCHK(g->bin_dist.alloc(std::max<int64_t>(n, 1) * 32));
    HIPCHK(g->attrs.alloc(std::max<int64_t>(n, 1) * 3));
    HIPCHK(g->gridconn.alloc(std::max<int64_t>(n, 1)));

    // capacities (retried on overflow)
    // LDS gap / block lists: small lists keep the per-wave LDS near 12 KB at 1000^2 (13 waves per CU
    // instead of 10 with 64-entry lists: 8.27 s -> 6.6 s); longer block lists spill to HBM, longer gap
    // lists re-run the source with larger capacities
    int gcap = MK_GCAP0, bcap = MK_BCAP0;
    int spill_cap = 4096;      // per-wave HBM blocks past bcap
    int64_t capB = 32 * (int64_t)D + 2048;
    if (const char* e = getenv("DMX_MK_GCAP")) gcap = std::max(2, atoi(e));   // test hooks for the retry path
    if (const char* e = getenv("DMX_MK_BCAP")) bcap = std::max(2, atoi(e));
    if (const char* e = getenv("DMX_MK_SPILL")) spill_cap = std::max(1, atoi(e));
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    const int64_t n_src = only ? (int64_t)only->size() : n;   // sources this call sweeps
    if (only)
        for (int64_t v : *only)
            if (v < node_begin || v >= node_end) return fail(DMX_ERR_ARG, "sample node outside the range");
    int64_t pool_cap = std::max<int64_t>(n_src * std::max<int64_t>(64, 6 * (int64_t)D), 1024);
    // A whole-graph build does the VGA symmetry certificate's scatter as it publishes each source's runs
    // (the runs are in the L2 then, and the memory-side atomics overlap the sweep), instead of a later pass
    // over the 36 GB pool (0.38 s at 1000^2).  Ranges, samples and cost counts leave it to prepare_symmetry.
    const bool fuse_sym = !only && d_work == nullptr && node_begin == 0 && node_end == N && N > 0 &&
                          !getenv("DMX_MK_NOSYM");
    const int64_t Cc = (int64_t)h.cols() * h.rows();
    if (fuse_sym) {
        HIPCHK(g->sym_prefix.alloc((size_t)4 * Cc));
        HIPCHK(g->sym_diff.alloc((size_t)4 * Cc));
        HIPCHK(g->sym_ho.alloc(N));
        const int maxlines = h.cols() + h.rows();
        hipLaunchKernelGGL(sym_lines_kernel, dim3((maxlines + 127) / 128, 4), dim3(128), 0, ctx->stream, h.cols(),
                           h.rows(), pm->d_cell_node.p, g->sym_prefix.p, 0);
        HIPCHK(hipGetLastError());
    }
    ctx->last_mk_s = 0;
    double sqrt_err = 0.0;
    if (int rc2 = mk_sqrt_err(ctx, 2ll * D * D, &sqrt_err)) return rc2;
    DevBuf<int64_t> fail_list, node_list;
    DevBuf<MakeGraphParams> dP;   // kernel parameters in device memory (see makegraph_kernel)
    HIPCHK(fail_list.alloc(std::max<int64_t>(n, 1)));
    HIPCHK(node_list.alloc(std::max<int64_t>(n, 1)));
    // Run pool size.  The worst case above (6 runs per depth per source) is ~1.4x the real count at
    // 1000^2; at 2000^2 it exceeds the device, and clamping it to the free memory would leave nothing
    // for the scan order a following VGA needs.  When the worst case takes more than 40 % of the free
    // memory, a first pass over an evenly spaced sample of sources measures the runs per source and
    // the pool takes 1.25x that plus 64 per source (0.08 s at 1000^2, so skipped there).  An overflow
    // still re-runs everything with a doubled pool.
    const int64_t kSample = 4096;
    const bool big_pool = (double)pool_cap * sizeof(Run) > 0.4 * (double)(free_b + cached_bytes());
    bool sampling = !only && !getenv("DMX_MK_NOSAMPLE") &&
                    ((n >= 16 * kSample && big_pool) || (n >= kSample && getenv("DMX_MK_SAMPLE")));   // test hook
    double mk_total_s = 0.0;
    int64_t reruns = 0;   // sources re-run after a first-pass capacity or certification failure
    std::vector<int64_t> mk_reruns;
    for (int restart = 0; restart < 4; restart++) {
        // one full pass, then re-runs of only the sources that overflowed an LDS / staging capacity
        double kernel_s = 0.0;
        int64_t list_n = -1;   // -1: the whole range
        if (only) {
            list_n = n_src;
            if (list_n)
                HIPCHK(hipMemcpyAsync(node_list.p, only->data(), list_n * 8, hipMemcpyHostToDevice, ctx->stream));
        }
        bool pool_over = false;
        const int64_t pool_cap_full = pool_cap;
        if (fuse_sym) {   // every pass publishes each source once; a restarted pass starts over
            HIPCHK(hipMemsetAsync(g->sym_diff.p, 0, (size_t)4 * Cc * 8, ctx->stream));
            HIPCHK(hipMemsetAsync(g->sym_ho.p, 0, (size_t)N * 8, ctx->stream));
        }
        if (sampling) {
            std::vector<int64_t> sl((size_t)kSample);
            for (int64_t i = 0; i < kSample; i++) sl[i] = node_begin + (i * n) / kSample + n / (2 * kSample);
            HIPCHK(hipMemcpyAsync(node_list.p, sl.data(), kSample * 8, hipMemcpyHostToDevice, ctx->stream));
            list_n = kSample;
            pool_cap = kSample * std::max<int64_t>(64, 6 * (int64_t)D);
        }
        HIPCHK(hipMemsetAsync(ctx->counters.p, 0, 16 * sizeof(int), ctx->stream));
        HIPCHK(hipMemsetAsync(ctx->stats.p, 0, 32 * sizeof(unsigned long long), ctx->stream));
        size_t lds0 = makegraph_lds(gcap, bcap, D);
        int occ0 = 0;
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ0, mk_kernel(false, d_work != nullptr, false, false), 64, lds0));
        {
            const int64_t waves0 = std::min<int64_t>((int64_t)ctx->num_cu * std::max(occ0, 1), std::max<int64_t>(n, 1));
            const size_t stage0 = (size_t)waves0 * (capB * 16 + (3 * ((size_t)D + 1) + 4) * 4) * 4;   // headroom for retries
            HIPCHK(hipMemGetInfo(&free_b, &total_b));
            free_b += cached_bytes();   // released by cached_malloc if the fresh allocation needs them
            const size_t pool_bytes_max = free_b > stage0 + (1ull << 30) ? (free_b - stage0 - (1ull << 30)) : 0;
            if ((size_t)pool_cap * sizeof(Run) > pool_bytes_max) pool_cap = (int64_t)(pool_bytes_max / sizeof(Run));
            if (pool_cap <= 0) return fail(DMX_ERR_HIP, "not enough device memory for the run pool");
            double ta = now_s();
            HIPCHK(g->pool.alloc(pool_cap));
            VLOG("makegraph: pool alloc %.3f GB %.3f s\n", pool_cap * 8.0 / 1e9, now_s() - ta);
        }
        for (int attempt = 0; attempt < 8; attempt++) {
            size_t lds = makegraph_lds(gcap, bcap, D);
            if (lds > 160 * 1024) return fail(DMX_ERR_CAPACITY, "makegraph LDS requirement exceeds 160 KiB");
            // re-runs (and every pass when the device square root is not accurate enough): the serial moment chains
            const bool exact_pass = attempt > 0 || getenv("DMX_MK_EXACT") || !(sqrt_err < 0x1p-30) || getenv("DMX_MK_SQRT_BAD");
            const mk_kernel_t kern = mk_kernel(gcap == MK_GCAP0 && bcap == MK_BCAP0 && !exact_pass &&
                                                   !getenv("DMX_MK_NOFIXED"),
                                               d_work != nullptr, maxdist != -1.0, D + 4 > MK_OPEN_LDS);
            int occ = 0;
            HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, 64, lds));
            if (occ < 1) occ = 1;
            const int64_t todo = list_n < 0 ? n : list_n;
            const int64_t waves = std::min<int64_t>((int64_t)ctx->num_cu * occ, std::max<int64_t>(todo, 1));
            const int64_t capA = capB;
            DevBuf<unsigned long long> stA;
            DevBuf<Run> stB;
            DevBuf<uint32_t> pref, rcnt;
            HIPCHK(stA.alloc((size_t)waves * capA));
            HIPCHK(stB.alloc((size_t)waves * capB));
            HIPCHK(pref.alloc((size_t)waves * (3 * ((size_t)D + 1) + 4)));
            HIPCHK(rcnt.alloc((size_t)waves * (3 * ((size_t)D + 1) + 4)));
            HIPCHK(hipMemsetAsync(rcnt.p, 0, (size_t)waves * (3 * ((size_t)D + 1) + 4) * 4, ctx->stream));
            const int openh_n = std::max(0, D + 4 - MK_OPEN_LDS);
            DevBuf<uint32_t> openh;
            HIPCHK(openh.alloc(std::max<size_t>((size_t)waves * openh_n, 1)));
            HIPCHK(hipMemsetAsync(openh.p, 0, std::max<size_t>((size_t)waves * openh_n, 1) * 4, ctx->stream));
            DevBuf<double2> bsp;
            DevBuf<int> bspf;
            HIPCHK(bsp.alloc((size_t)waves * 2 * spill_cap));
            HIPCHK(bspf.alloc((size_t)waves * spill_cap));
            // work counter, error word and failure count restart; the pool cursor carries on
            HIPCHK(hipMemsetAsync(ctx->counters.p, 0, 2 * sizeof(int), ctx->stream));
            HIPCHK(hipMemsetAsync(ctx->counters.p + 4, 0, sizeof(int), ctx->stream));
            MakeGraphParams P;
            P.cols = h.cols(); P.rows = h.rows();
            P.spacing = h.spacing(); P.blx = h.bottom_left().x; P.bly = h.bottom_left().y;
            P.maxdist = maxdist;
            P.cellw = pm->d_cellw.p; P.segs = pm->d_segs.p; P.node_cell = pm->d_node_cell.p;
            P.sqrt_err = sqrt_err;
            P.node_begin = node_begin; P.node_end = node_end;
            P.work_counter = ctx->counters.p + 0;
            P.ctl = ctx->d_ctl;
            ctx->h_ctl->progress = 0;
            P.error = ctx->counters.p + 1;
            P.pool_cursor = (unsigned long long*)(ctx->counters.p + 2);
            P.pool_capacity = pool_cap; P.pool = g->pool.p;
            P.node_run_start = g->node_run_start.p; P.bin_nruns = g->bin_nruns.p; P.bin_count = g->bin_count.p;
            P.bin_dist = g->bin_dist.p; P.attrs = g->attrs.p;
            P.stageA = stA.p; P.stageB = stB.p; P.prefix = pref.p; P.runcnt = rcnt.p;
            P.capA = (int)capA; P.capB = (int)capB; P.gcap = gcap; P.bcap = bcap; P.dmax = D;
            P.bspill = bsp.p; P.bspill_flag = bspf.p; P.spill_cap = spill_cap;
            P.stats = ctx->stats.p;
            P.node_list = list_n < 0 ? nullptr : node_list.p;
            P.list_n = list_n < 0 ? 0 : list_n;
            P.fail_list = fail_list.p;
            P.fail_count = ctx->counters.p + 4;
            P.profile = verbose() ? 1 : 0;
            // the first pass certifies parallel moment sums; re-runs of failed sources use the serial chains
            P.exact_moments = exact_pass ? 1 : 0;
            P.src_work = d_work;
            P.openh = openh.p; P.openh_n = openh_n;
            const bool sym_pass = fuse_sym && !sampling;   // the sampling pass's runs are thrown away
            P.sym_prefix = sym_pass ? g->sym_prefix.p : nullptr;
            P.sym_diff = sym_pass ? g->sym_diff.p : nullptr;
            P.sym_ho = sym_pass ? g->sym_ho.p : nullptr;
            // the shortest span taken (DMX_MK_SPAN: A/B hook; DMX_MK_NOSPAN: every depth cell by cell)
            P.spans = getenv("DMX_MK_NOSPAN") ? 0 : (getenv("DMX_MK_SPAN") ? std::max(1, atoi(getenv("DMX_MK_SPAN"))) : MK_SPAN_MIN);
            HIPCHK(hipEventRecord(ctx->ev0, ctx->stream));
            if (todo > 0) {
                HIPCHK(dP.alloc(1));
                HIPCHK(hipMemcpyAsync(dP.p, &P, sizeof(P), hipMemcpyHostToDevice, ctx->stream));
                hipLaunchKernelGGL(kern, dim3((unsigned)waves), dim3(64), lds, ctx->stream,
                                   (const MakeGraphParams*)dP.p);
                HIPCHK(hipGetLastError());
            }
            HIPCHK(hipEventRecord(ctx->ev1, ctx->stream));
            HIPCHK(wait_progress(ctx, DMX_PHASE_MAKEGRAPH, todo, 1));
            CANCEL_POINT(ctx);
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
            kernel_s += ms * 1e-3;
            int hc[5] = {0, 0, 0, 0, 0};
            HIPCHK(copy_sync(ctx->stream, hc, ctx->counters.p, sizeof(hc), hipMemcpyDeviceToHost));
            const int err = hc[1], nfail = hc[4];
            VLOG("makegraph: attempt %d (%lld sources, gcap %d bcap %d spill %d capB %lld, occupancy %d): %.3f s, %d failed, "
                 "err %d\n", attempt, (long long)todo, gcap, bcap, spill_cap, (long long)capB, occ, ms * 1e-3, nfail, err);
            if (err & KERR_BIN_MISMATCH) return fail(DMX_ERR_STATE, "internal: whichbin outside octant");
            if (err & KERR_POOL_CAPACITY) {
                unsigned long long used = 0;
                std::memcpy(&used, &hc[2], 8);
                pool_cap = std::max<int64_t>(pool_cap * 2, (int64_t)used + 1024);
                pool_over = true;
                break;
            }
            if (nfail == 0) break;
            if (!sampling) {
                reruns += nfail;
                std::vector<int64_t> fl((size_t)nfail);
                HIPCHK(copy_sync(ctx->stream, fl.data(), fail_list.p, (size_t)nfail * 8, hipMemcpyDeviceToHost));
                mk_reruns.insert(mk_reruns.end(), fl.begin(), fl.end());
            }
            if (err & KERR_GAP_CAPACITY) gcap *= 2;
            if (err & KERR_BLOCK_CAPACITY) spill_cap *= 4;
            if (err & KERR_STAGE_CAPACITY) capB *= 2;
            HIPCHK(hipMemcpyAsync(node_list.p, fail_list.p, (size_t)nfail * 8, hipMemcpyDeviceToDevice, ctx->stream));
            list_n = nfail;
            if (attempt == 7) return fail(DMX_ERR_CAPACITY, "makegraph capacities exceeded after retries");
        }
        if (sampling) {
            unsigned long long used = 0;
            HIPCHK(copy_sync(ctx->stream, &used, ctx->counters.p + 2, 8, hipMemcpyDeviceToHost));
            sampling = false;
            mk_total_s += kernel_s;
            if (pool_over) { pool_cap = pool_cap_full; continue; }   // no estimate: the worst-case pool
            const double per_src = (double)used / (double)kSample;
            pool_cap = std::min<int64_t>(pool_cap_full, (int64_t)(1.25 * per_src * (double)n) + 64 * n + 4096);
            VLOG("makegraph: sample of %lld sources, %.1f runs each -> pool %.3f GB\n", (long long)kSample, per_src,
                 pool_cap * 8.0 / 1e9);
            continue;
        }
        if (pool_over) { mk_total_s += kernel_s; mk_reruns.clear(); reruns = 0; continue; }
        HIPCHK(hipEventRecord(ctx->ev0, ctx->stream));
        if (n > 0 && !only) {   // (a sample leaves the other nodes' run starts unset)
            hipLaunchKernelGGL(gridconn_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, h.rows(),
                               pm->d_node_cell.p + node_begin, n, g->node_run_start.p, g->bin_nruns.p, g->pool.p,
                               g->gridconn.p);
            HIPCHK(hipGetLastError());
            hipLaunchKernelGGL(node_nruns_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream,
                               g->bin_nruns.p, n, g->node_nruns.p);
            HIPCHK(hipGetLastError());
        }
        HIPCHK(hipEventRecord(ctx->ev1, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
        kernel_s += ms * 1e-3;
        int hc[4] = {0, 0, 0, 0};
        HIPCHK(copy_sync(ctx->stream, hc, ctx->counters.p, sizeof(hc), hipMemcpyDeviceToHost));
        unsigned long long used = 0;
        std::memcpy(&used, &hc[2], 8);
        unsigned long long st[26];
        HIPCHK(copy_sync(ctx->stream, st, ctx->stats.p, sizeof(st), hipMemcpyDeviceToHost));
        if (verbose()) {
            double tot = (double)st[22];
            for (int i = 8; i < 18; i++) tot += (double)st[i];
            VLOG("makegraph phases (wave clocks): garbage %.1f%%, ranges %.1f%%, candidates %.1f%%, bins %.1f%%, "
                 "moments %.1f%%, run tracking %.1f%%, placement %.1f%%, publish %.1f%%, depth tail %.1f%%, "
                 "octant setup %.1f%% (%.3g total; %llu depth steps, %llu chunks, %llu candidates)\n", 100 * st[8] / tot,
                 100 * st[9] / tot, 100 * st[10] / tot, 100 * st[11] / tot, 100 * st[12] / tot, 100 * st[13] / tot,
                 100 * st[14] / tot, 100 * st[15] / tot, 100 * st[16] / tot, 100 * st[17] / tot, tot, st[2], st[3], st[0]);
            VLOG("makegraph merges: %llu (%llu with one block), %.2f blocks and %.2f gaps a merge\n", st[18], st[19],
                 st[18] ? (double)st[20] / st[18] : 0.0, st[18] ? (double)st[21] / st[18] : 0.0);
            VLOG("makegraph spans: %.1f%% of the clocks; %llu spans over %llu depths (%.1f each), %llu of %llu visible cells "
                 "(%.1f%%)\n", 100 * st[22] / tot, st[23], st[24], st[23] ? (double)st[24] / st[23] : 0.0, st[25], st[1],
                 st[1] ? 100.0 * st[25] / st[1] : 0.0);
        }
        ctx->last_stats[0] = (long long)st[0];
        ctx->last_stats[1] = (long long)st[1];
        ctx->last_stats[2] = (long long)used;
        ctx->last_stats[32] = (long long)st[2];   // sieve depth steps
        ctx->last_stats[33] = (long long)st[3];   // 64-candidate chunks
        ctx->last_stats[34] = (long long)reruns;
        ctx->last_mk_reruns = std::move(mk_reruns);
        ctx->last_mk_s = mk_total_s + kernel_s;   // every pass counted (sample, overflow re-runs)
        g->nruns = (int64_t)used;
        if (fuse_sym) { g->sym_fused = true; g->sym_prefix.reset(); }   // the prefix sums are no longer needed
        VLOG("makegraph: kernels %.3f s, total %.3f s\n", kernel_s, now_s() - t_start);
        *out = g.release();
        return DMX_OK;
    }
    return fail(DMX_ERR_CAPACITY, "makegraph capacities exceeded after retries");
}

int dmx_makegraph(dmx_ctx* ctx, dmx_pointmap* pm, double maxdist, int boundary, int64_t node_begin, int64_t node_end,
                  dmx_graph** out) {
    return makegraph_impl(ctx, pm, maxdist, boundary, node_begin, node_end, nullptr, nullptr, out);
}

// Cost model of one source's sweep, in units of one depth step: a source pays a fixed setup, one unit per
// sieve depth step (collectgarbage + visit ranges) and kMkChunkCost per 64-candidate chunk (tests, bins,
// moments, run tracking).  Fitted to per-strip kernel times on MI355X.
static const double kMkSourceCost = 0.0, kMkChunkCost = 0.7;

int dmx_makegraph_balance(dmx_ctx* ctx, dmx_pointmap* pm, double maxdist, int boundary, int32_t world, int64_t stride,
                          int64_t* bounds) {
    if (!ctx || !pm || !bounds || world < 1 || stride < 1) return fail(DMX_ERR_ARG, "bad arguments");
    HIPCHK(hipSetDevice(ctx->device));
    PointMapHost& h = *pm->host;
    if (!h.lines_blocked()) h.block_lines();
    if (boundary) { h.keep_edges_only(); pm->version++; }
    int rc = upload_pointmap(ctx, pm);
    if (rc) return rc;
    const int64_t N = pm->nnodes;
    bounds[0] = 0;
    for (int r = 1; r <= world; r++) bounds[r] = N;
    if (N == 0 || world == 1) return DMX_OK;
    // sample j stands for the nodes [j*stride, (j+1)*stride): its middle node is swept
    const int64_t ns = (N + stride - 1) / stride;
    std::vector<int64_t> sample((size_t)ns);
    for (int64_t j = 0; j < ns; j++) sample[j] = std::min<int64_t>(N - 1, j * stride + stride / 2);
    DevBuf<uint32_t> d_work;
    HIPCHK(d_work.alloc((size_t)N * 2));
    HIPCHK(hipMemsetAsync(d_work.p, 0xFF, (size_t)N * 2 * 4, ctx->stream));   // unwritten entries stay ~0u
    dmx_graph* g = nullptr;
    rc = makegraph_impl(ctx, pm, maxdist, 0, 0, N, &sample, d_work.p, &g);   // boundary already applied
    if (rc) return rc;
    dmx_graph_free(g);
    std::vector<uint32_t> w2((size_t)N * 2);
    HIPCHK(copy_sync(ctx->stream, w2.data(), d_work.p, (size_t)N * 2 * 4, hipMemcpyDeviceToHost));
    // cumulative modelled cost at the interval ends; bounds at equal shares (same doubles on every rank)
    std::vector<double> cum((size_t)ns + 1, 0.0);
    for (int64_t j = 0; j < ns; j++) {
        const int64_t v = sample[j];
        if (w2[2 * v] == ~0u || w2[2 * v + 1] == ~0u)
            return fail(DMX_ERR_STATE, "internal: the makeGraph cost sample did not record every sampled source");
        const double w = kMkSourceCost + (double)w2[2 * v] + kMkChunkCost * (double)w2[2 * v + 1];
        const int64_t cnt = std::min<int64_t>(N, (j + 1) * stride) - j * stride;
        cum[j + 1] = cum[j] + w * (double)cnt;
    }
    int64_t j = 0;
    for (int r = 1; r < world; r++) {
        const double target = cum[ns] * (double)r / (double)world;
        while (j < ns - 1 && cum[j + 1] < target) j++;
        const double per = (cum[j + 1] - cum[j]) / (double)(std::min<int64_t>(N, (j + 1) * stride) - j * stride);
        int64_t b = j * stride + (per > 0.0 ? (int64_t)((target - cum[j]) / per) : 0);
        b = std::max<int64_t>(b, bounds[r - 1]);
        bounds[r] = std::min<int64_t>(b, N);
    }
    return DMX_OK;
}

int dmx_graph_free(dmx_graph* g) {
    if (g && g->ctx) (void)hipSetDevice(g->ctx->device);
    delete g;
    return DMX_OK;
}

int dmx_graph_info(const dmx_graph* g, int64_t* nnodes, int64_t* nb, int64_t* ne, int64_t* nruns) {
    if (!g) return fail(DMX_ERR_ARG, "graph is NULL");
    if (nnodes) *nnodes = g->nnodes;
    if (nb) *nb = g->node_begin;
    if (ne) *ne = g->node_end;
    if (nruns) *nruns = g->nruns;
    return DMX_OK;
}

int dmx_graph_copy_range(dmx_graph* g, int64_t kb, int64_t ke, float* attrs, int32_t* bins, int16_t* runs,
                         int64_t runs_cap, int64_t* nruns_out, uint8_t* gridconn) {
    if (!g) return fail(DMX_ERR_ARG, "graph is NULL");
    const int64_t nl = g->node_end - g->node_begin;
    if (ke < 0) ke = nl;
    if (kb < 0 || kb > ke || ke > nl) return fail(DMX_ERR_ARG, "node range outside the graph");
    HIPCHK(hipSetDevice(g->ctx->device));
    hipStream_t st = g->ctx->stream;
    const int64_t n = ke - kb;
    if (nruns_out) *nruns_out = 0;
    if (n == 0) return DMX_OK;
    if (attrs) HIPCHK(copy_sync(st, attrs, g->attrs.p + kb * 3, n * 3 * 4, hipMemcpyDeviceToHost));
    if (gridconn) HIPCHK(copy_sync(st, gridconn, g->gridconn.p + kb, n, hipMemcpyDeviceToHost));
    std::vector<int32_t> bn((size_t)n * 32);
    HIPCHK(copy_sync(st, bn.data(), g->bin_nruns.p + kb * 32, n * 32 * 4, hipMemcpyDeviceToHost));
    if (bins) {
        std::vector<uint16_t> bc((size_t)n * 32);
        std::vector<float> bd((size_t)n * 32);
        HIPCHK(copy_sync(st, bc.data(), g->bin_count.p + kb * 32, n * 32 * 2, hipMemcpyDeviceToHost));
        HIPCHK(copy_sync(st, bd.data(), g->bin_dist.p + kb * 32, n * 32 * 4, hipMemcpyDeviceToHost));
        for (int64_t k = 0; k < n; k++)
            for (int b = 0; b < 32; b++) {
                const int64_t i = k * 32 + b;
                int dir; // Node::make (ngraph.cpp:43-54); empty bins keep NODIR
                if (b == 4 || b == 20) dir = 4;
                else if (b == 12 || b == 28) dir = 8;
                else if ((b > 4 && b < 12) || (b > 20 && b < 28)) dir = 2;
                else dir = 1;
                bins[i * 4 + 0] = bn[i] > 0 ? dir : 0;
                bins[i * 4 + 1] = bc[i];
                std::memcpy(&bins[i * 4 + 2], &bd[i], 4);
                bins[i * 4 + 3] = bn[i];
            }
    }
    int64_t acc = 0;
    std::vector<int64_t> dst((size_t)n);
    for (int64_t k = 0; k < n; k++) {
        int sum = 0;
        for (int b = 0; b < 32; b++) sum += bn[k * 32 + b];
        dst[k] = acc;
        acc += sum;
    }
    if (nruns_out) *nruns_out = acc;
    if (runs) {
        if (runs_cap >= 0 && acc > runs_cap) return fail(DMX_ERR_ARG, "runs buffer too small for the node range");
        // node-ordered copy (the pool is in completion order), gathered in node batches of at most
        // kChunk runs so that the staging buffer stays small next to a 90 GB graph
        const int64_t kChunk = (int64_t)1 << 29;   // 4 GiB of runs
        DevBuf<int64_t> d_dst;
        DevBuf<Run> d_runs;
        HIPCHK(d_dst.alloc(n));
        HIPCHK(d_runs.alloc(std::max<int64_t>(std::min(acc, kChunk), 1)));
        int64_t k0 = 0;
        while (k0 < n) {
            int64_t k1 = k0;
            const int64_t base = dst[k0];
            while (k1 < n && (k1 == k0 || (k1 + 1 < n ? dst[k1 + 1] : acc) - base <= kChunk)) k1++;
            const int64_t cnt = (k1 < n ? dst[k1] : acc) - base;
            std::vector<int64_t> rel((size_t)(k1 - k0));
            for (int64_t k = k0; k < k1; k++) rel[k - k0] = dst[k] - base;
            if (cnt > (int64_t)d_runs.n) HIPCHK(d_runs.alloc(cnt));   // one node above the chunk size
            HIPCHK(copy_sync(st, d_dst.p, rel.data(), (k1 - k0) * 8, hipMemcpyHostToDevice));
            hipLaunchKernelGGL(gather_runs_kernel, dim3((unsigned)(k1 - k0)), dim3(256), 0, st, g->pool.p,
                               g->node_run_start.p + kb + k0, g->node_nruns.p + kb + k0, d_dst.p, k1 - k0, d_runs.p);
            HIPCHK(hipGetLastError());
            if (cnt) HIPCHK(copy_sync(st, runs + base * 4, d_runs.p, cnt * sizeof(Run), hipMemcpyDeviceToHost));
            k0 = k1;
        }
    }
    return DMX_OK;
}

int dmx_graph_copy(dmx_graph* g, float* attrs, int32_t* bins, int16_t* runs, uint8_t* gridconn) {
    return dmx_graph_copy_range(g, 0, -1, attrs, bins, runs, -1, nullptr, gridconn);
}

// ---------------------------------------------------------------- shard blobs
// layout: int64 header[4] {node_begin, node_end, nruns, magic}, then (8-byte aligned sections)
// bin_nruns i32[n*32], bin_count u16[n*32], bin_dist f32[n*32], attrs f32[n*3], gridconn u8[n],
// runs (node order).
static const int64_t kBlobMagic = 0x31424d58444d44LL;
static inline int64_t al8(int64_t x) { return (x + 7) & ~7LL; }
static void blob_layout(int64_t n, int64_t nruns, int64_t* off /*7*/) {
    off[0] = 32;
    off[1] = off[0] + al8(n * 32 * 4);
    off[2] = off[1] + al8(n * 32 * 2);
    off[3] = off[2] + al8(n * 32 * 4);
    off[4] = off[3] + al8(n * 3 * 4);
    off[5] = off[4] + al8(n);
    off[6] = off[5] + nruns * 8;
}

int dmx_graph_blob_size(dmx_graph* g, int64_t* bytes) {
    if (!g || !bytes) return fail(DMX_ERR_ARG, "bad arguments");
    int64_t off[7];
    blob_layout(g->node_end - g->node_begin, g->nruns, off);
    *bytes = off[6];
    return DMX_OK;
}

int dmx_graph_blob_write_device(dmx_graph* g, void* dst, int64_t bytes) {
    if (!g || !dst) return fail(DMX_ERR_ARG, "bad arguments");
    HIPCHK(hipSetDevice(g->ctx->device));
    const int64_t n = g->node_end - g->node_begin;
    int64_t off[7];
    blob_layout(n, g->nruns, off);
    if (bytes < off[6]) return fail(DMX_ERR_ARG, "blob buffer too small");
    char* d = (char*)dst;
    hipStream_t s = g->ctx->stream;
    int64_t hdr[4] = {g->node_begin, g->node_end, g->nruns, kBlobMagic};
    HIPCHK(hipMemcpyAsync(d, hdr, 32, hipMemcpyHostToDevice, s));
    if (n) {
        HIPCHK(hipMemcpyAsync(d + off[0], g->bin_nruns.p, n * 32 * 4, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(d + off[1], g->bin_count.p, n * 32 * 2, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(d + off[2], g->bin_dist.p, n * 32 * 4, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(d + off[3], g->attrs.p, n * 3 * 4, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(d + off[4], g->gridconn.p, n, hipMemcpyDeviceToDevice, s));
        std::vector<int32_t> nr((size_t)n);
        HIPCHK(hipMemcpyAsync(nr.data(), g->node_nruns.p, n * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        std::vector<int64_t> dsto((size_t)n);
        int64_t acc = 0;
        for (int64_t k = 0; k < n; k++) { dsto[k] = acc; acc += nr[k]; }
        DevBuf<int64_t> d_dst;
        HIPCHK(d_dst.alloc(n));
        HIPCHK(hipMemcpyAsync(d_dst.p, dsto.data(), n * 8, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(gather_runs_kernel, dim3((unsigned)n), dim3(256), 0, s, g->pool.p, g->node_run_start.p,
                           g->node_nruns.p, d_dst.p, n, (Run*)(d + off[5]));
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(s));
    return DMX_OK;
}

int dmx_graph_assemble_device(dmx_ctx* ctx, dmx_pointmap* pm, const void* const* blobs, const int64_t* sizes,
                              int nshards, dmx_graph** out) {
    if (!ctx || !pm || !blobs || !out || nshards <= 0) return fail(DMX_ERR_ARG, "bad arguments");
    HIPCHK(hipSetDevice(ctx->device));
    int rc = upload_pointmap(ctx, pm);
    if (rc) return rc;
    const int64_t N = pm->nnodes;
    std::vector<std::array<int64_t, 4>> hdr((size_t)nshards);
    int64_t total_runs = 0;
    for (int i = 0; i < nshards; i++) {
        HIPCHK(copy_sync(ctx->stream, hdr[i].data(), blobs[i], 32, hipMemcpyDeviceToHost));
        if (hdr[i][3] != kBlobMagic) return fail(DMX_ERR_ARG, "not a dmx graph blob");
        total_runs += hdr[i][2];
    }
    std::unique_ptr<dmx_graph> g(new dmx_graph());
    g->ctx = ctx; g->pm = pm; g->nnodes = N; g->node_begin = 0; g->node_end = N; g->nruns = total_runs;
    inherit_merges(g.get());
    HIPCHK(g->node_run_start.alloc(std::max<int64_t>(N, 1)));
    HIPCHK(g->node_nruns.alloc(std::max<int64_t>(N, 1)));
    HIPCHK(g->bin_nruns.alloc(std::max<int64_t>(N, 1) * 32));
    HIPCHK(g->bin_count.alloc(std::max<int64_t>(N, 1) * 32));
    HIPCHK(g->bin_dist.alloc(std::max<int64_t>(N, 1) * 32));
    HIPCHK(g->attrs.alloc(std::max<int64_t>(N, 1) * 3));
    HIPCHK(g->gridconn.alloc(std::max<int64_t>(N, 1)));
    HIPCHK(g->pool.alloc(std::max<int64_t>(total_runs, 1)));
    hipStream_t s = ctx->stream;
    std::vector<char> covered((size_t)N, 0);
    // shards are placed in node order; runs of a shard are contiguous in node order
    std::vector<int> order(nshards);
    for (int i = 0; i < nshards; i++) order[i] = i;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return hdr[a][0] < hdr[b][0]; });
    int64_t run_base = 0;
    for (int oi = 0; oi < nshards; oi++) {
        const int i = order[oi];
        const int64_t b = hdr[i][0], e = hdr[i][1], n = e - b, nr = hdr[i][2];
        if (b < 0 || e > N || b > e) return fail(DMX_ERR_ARG, "blob node range does not fit the point map");
        int64_t off[7];
        blob_layout(n, nr, off);
        if (sizes && sizes[i] < off[6]) return fail(DMX_ERR_ARG, "blob shorter than its header says");
        for (int64_t k = b; k < e; k++) {
            if (covered[k]) return fail(DMX_ERR_ARG, "overlapping shards");
            covered[k] = 1;
        }
        const char* d = (const char*)blobs[i];
        if (n) {
            HIPCHK(hipMemcpyAsync(g->bin_nruns.p + b * 32, d + off[0], n * 32 * 4, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipMemcpyAsync(g->bin_count.p + b * 32, d + off[1], n * 32 * 2, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipMemcpyAsync(g->bin_dist.p + b * 32, d + off[2], n * 32 * 4, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipMemcpyAsync(g->attrs.p + b * 3, d + off[3], n * 3 * 4, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipMemcpyAsync(g->gridconn.p + b, d + off[4], n, hipMemcpyDeviceToDevice, s));
        }
        if (nr) HIPCHK(hipMemcpyAsync(g->pool.p + run_base, d + off[5], nr * 8, hipMemcpyDeviceToDevice, s));
        run_base += nr;
    }
    for (int64_t k = 0; k < N; k++)
        if (!covered[k]) return fail(DMX_ERR_ARG, "shards do not cover every node");
    if (N) {
        hipLaunchKernelGGL(node_nruns_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, g->bin_nruns.p, N,
                           g->node_nruns.p);
        HIPCHK(hipGetLastError());
        std::vector<int32_t> nr((size_t)N);
        HIPCHK(hipMemcpyAsync(nr.data(), g->node_nruns.p, N * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        std::vector<int64_t> st((size_t)N);
        int64_t acc = 0;
        for (int64_t k = 0; k < N; k++) { st[k] = acc; acc += nr[k]; }
        if (acc != total_runs) return fail(DMX_ERR_ARG, "blob run counts inconsistent");
        HIPCHK(hipMemcpyAsync(g->node_run_start.p, st.data(), N * 8, hipMemcpyHostToDevice, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    *out = g.release();
    return DMX_OK;
}

// ---------------------------------------------------------------- VGA global
// Node range of this rank's share of the preparation scatters ([0, N) when not sharded).
static void prep_range(const dmx_graph* g, int64_t& b, int64_t& e) {
    b = 0; e = g->nnodes;
    if (g->prep_fn && g->prep_e >= 0) { b = g->prep_b; e = g->prep_e; }
}
// Sum a partial device buffer over the ranks (no-op when not sharded).  The stream is drained first:
// the caller's collective runs on its own stream and returns only once the sum is in place.
static int prep_allreduce(dmx_graph* g, void* p, int64_t count, int dtype) {
    if (!g->prep_fn || count <= 0) return DMX_OK;
    HIPCHK(hipStreamSynchronize(g->ctx->stream));
    if (g->prep_fn(p, count, dtype, g->prep_user) != 0)
        return fail(DMX_ERR_STATE, "prep all-reduce callback failed");
    return DMX_OK;
}
// U_f (filled cells that appear in some run: the early-exit universe of every BFS) by range counts,
// plus the longest-first scan pool.  O(runs) with a few line-prefix passes.
static int prepare_symmetry(dmx_graph* g);
static int build_scan_order(dmx_graph* g);
static int prepare_uf(dmx_graph* g) {
    if (g->scan_ready) return DMX_OK;
    // the symmetry pass computes U_f from its in-set hashes; coverage counting only when it is skipped
    if (int rc = prepare_symmetry(g)) return rc;
    dmx_ctx* ctx = g->ctx;
    hipStream_t s = ctx->stream;
    PointMapHost& h = *g->pm->host;
    const int cols = h.cols(), rows = h.rows();
    const int tw = (cols + 7) / 8, th = (rows + 7) / 8;
    const int64_t C = (int64_t)cols * rows, N = g->nnodes;
    DevBuf<int> cov;
    DevBuf<unsigned long long> cnt;
    HIPCHK(cnt.alloc(1));
    HIPCHK(hipMemsetAsync(cnt.p, 0, 8, s));
    const bool have_uf = g->uf_count >= 0;
    if (!have_uf) {
        HIPCHK(cov.alloc((size_t)4 * C));
        HIPCHK(g->uf_tiles.alloc((size_t)tw * th));
        HIPCHK(g->notuf_tiles.alloc((size_t)tw * th));
        HIPCHK(hipMemsetAsync(cov.p, 0, (size_t)4 * C * 4, s));
        int64_t pb, pe;
        prep_range(g, pb, pe);
        if (pe > pb) {
            hipLaunchKernelGGL(cov_scatter_kernel, dim3((unsigned)std::min<int64_t>(pe - pb, 4096)), dim3(256), 0, s,
                               cols, rows, pe - pb, g->node_run_start.p + pb, g->node_nruns.p + pb, g->pool.p, cov.p);
            HIPCHK(hipGetLastError());
        }
        if (int rc = prep_allreduce(g, cov.p, (int64_t)4 * C, DMX_I32)) return rc;
        hipLaunchKernelGGL(cov_lines_kernel, dim3((cols + rows + 127) / 128, 4), dim3(128), 0, s, cols, rows, cov.p);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(cov_tiles_kernel, dim3((tw * th + 255) / 256), dim3(256), 0, s, cols, rows, tw, th,
                           g->pm->d_cell_node.p, cov.p, g->uf_tiles.p, g->notuf_tiles.p, cnt.p);
        HIPCHK(hipGetLastError());
    }
    unsigned long long ufc = have_uf ? (unsigned long long)g->uf_count : 0ull;
    if (!have_uf) HIPCHK(copy_sync(s, &ufc, cnt.p, 8, hipMemcpyDeviceToHost));
    if (int rc = build_scan_order(g)) return rc;
    g->uf_count = (int64_t)ufc;
    g->scan_ready = true;
    return DMX_OK;
}

// The scan order: every node's runs longest-first (scan_pool, node order), with per-node and per-cell starts.
static int build_scan_order(dmx_graph* g) {
    dmx_ctx* ctx = g->ctx;
    hipStream_t s = ctx->stream;
    PointMapHost& h = *g->pm->host;
    const int rows = h.rows();
    const int64_t C = (int64_t)h.cols() * rows, N = g->nnodes;
    std::vector<int32_t> nr((size_t)std::max<int64_t>(N, 1));
    if (N) HIPCHK(copy_sync(s, nr.data(), g->node_nruns.p, N * 4, hipMemcpyDeviceToHost));
    std::vector<int64_t> ss((size_t)std::max<int64_t>(N, 1));
    int64_t acc = 0;
    for (int64_t k = 0; k < N; k++) { ss[k] = acc; acc += nr[k]; }
    DevBuf<int64_t>& d_ss = g->scan_start;
    HIPCHK(d_ss.alloc(std::max<int64_t>(N, 1)));
    HIPCHK(g->scan_pool.alloc(std::max<int64_t>(acc, 1)));
    HIPCHK(g->cell_scan_start.alloc(C));
    HIPCHK(g->cell_nruns.alloc(C));
    HIPCHK(hipMemsetAsync(g->cell_nruns.p, 0, C * 4, s));
    if (N) {
        HIPCHK(hipMemcpyAsync(d_ss.p, ss.data(), N * 8, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(scan_pool_kernel, dim3((unsigned)std::min<int64_t>(N, 8192)), dim3(256), 0, s, rows,
                           g->pm->d_node_cell.p, N, g->node_run_start.p, g->node_nruns.p, g->bin_nruns.p, g->pool.p, d_ss.p,
                           g->scan_pool.p, g->cell_scan_start.p, g->cell_nruns.p);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(s));
    g->scan_released = false;
    return DMX_OK;
}

// The wide-grid partial-tile masks take the scan order's place (prepare_tiles): the searches that read the
// scan order itself (vga_do, a tile search without the masks) free the tile-visibility data and rebuild it.
static int restore_scan_order(dmx_graph* g) {
    if (!g->scan_released) return DMX_OK;
    g->pmask.reset(); g->ppre.reset(); g->poff.reset();
    g->tvis.reset(); g->ftvis.reset(); g->tvsum.reset(); g->tvnz.reset(); g->ttvis.reset();
    g->tvw = 0;
    g->tiles_ready = false;
    return build_scan_order(g);
}

// In-set corrections for bottom-up BFS (vga_do.hip, "symmetry / in-set corrections").
static int prepare_symmetry(dmx_graph* g) {
    if (g->symmetric >= 0) return DMX_OK;
    const char* force = getenv("DMX_VGA_KERNEL");
    if (force && std::string(force) == "topdown") {
        g->symmetric = 0;
        g->sym_diff.reset(); g->sym_ho.reset(); g->sym_fused = false;
        return DMX_OK;
    }
    dmx_ctx* ctx = g->ctx;
    hipStream_t s = ctx->stream;
    PointMapHost& h = *g->pm->host;
    const int cols = h.cols(), rows = h.rows();
    const int64_t C = (int64_t)cols * rows, N = g->nnodes;
    const int kSpecLimit = 4096;
    DevBuf<unsigned long long> prefix, diff_own, ho_own;
    DevBuf<int32_t> flist;
    DevBuf<int> fcount;
    HIPCHK(flist.alloc(kSpecLimit));
    HIPCHK(fcount.alloc(1));
    HIPCHK(hipMemsetAsync(fcount.p, 0, 4, s));
    const int maxlines = cols + rows;
    unsigned long long *diff = nullptr, *ho = nullptr;
    if (g->sym_fused) {
        // makeGraph did the scatter over the whole graph as it published the runs: complete on every rank,
        // so no all-reduce either
        diff = g->sym_diff.p;
        ho = g->sym_ho.p;
        ctx->last_stats[39] = 0;
    } else {
        const double t_sym = now_s();   // the scatter a sharded or assembled graph pays here (last_stats[39])
        HIPCHK(prefix.alloc((size_t)4 * C));
        HIPCHK(diff_own.alloc((size_t)4 * C));
        HIPCHK(ho_own.alloc(std::max<int64_t>(N, 1)));
        diff = diff_own.p;
        ho = ho_own.p;
        HIPCHK(hipMemsetAsync(diff, 0, (size_t)4 * C * 8, s));
        HIPCHK(hipMemsetAsync(ho, 0, (size_t)std::max<int64_t>(N, 1) * 8, s));
        hipLaunchKernelGGL(sym_lines_kernel, dim3((maxlines + 127) / 128, 4), dim3(128), 0, s, cols, rows,
                           g->pm->d_cell_node.p, prefix.p, 0);
        HIPCHK(hipGetLastError());
        int64_t pb, pe;
        prep_range(g, pb, pe);
        if (pe > pb) {
            hipLaunchKernelGGL(sym_scatter_kernel, dim3((unsigned)std::min<int64_t>(pe - pb, 4096)), dim3(256), 0, s,
                               cols, rows, g->pm->d_node_cell.p + pb, pe - pb, g->node_run_start.p + pb,
                               g->node_nruns.p + pb, g->pool.p, prefix.p, diff, ho + pb);
            HIPCHK(hipGetLastError());
        }
        if (int rc = prep_allreduce(g, diff, (int64_t)4 * C, DMX_I64)) return rc;
        if (int rc = prep_allreduce(g, ho, N, DMX_I64)) return rc;
        HIPCHK(hipStreamSynchronize(s));
        ctx->last_stats[39] = (long long)((now_s() - t_sym) * 1e6);
    }
    hipLaunchKernelGGL(sym_lines_kernel, dim3((maxlines + 127) / 128, 4), dim3(128), 0, s, cols, rows,
                       g->pm->d_cell_node.p, diff, 1);
    HIPCHK(hipGetLastError());
    if (N) {
        hipLaunchKernelGGL(sym_flag_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, rows,
                           g->pm->d_node_cell.p, N, C, diff, ho, fcount.p, flist.p, kSpecLimit);
        HIPCHK(hipGetLastError());
    }
    // U_f straight from the in-set hashes (uf_hi_tiles_kernel): no separate coverage pass
    const int tw = (cols + 7) / 8, th = (rows + 7) / 8;
    DevBuf<unsigned long long> ufcnt;
    HIPCHK(ufcnt.alloc(1));
    HIPCHK(hipMemsetAsync(ufcnt.p, 0, 8, s));
    HIPCHK(g->uf_tiles.alloc((size_t)tw * th));
    HIPCHK(g->notuf_tiles.alloc((size_t)tw * th));
    hipLaunchKernelGGL(uf_hi_tiles_kernel, dim3((tw * th + 255) / 256), dim3(256), 0, s, cols, rows, tw, th,
                       g->pm->d_cell_node.p, diff, g->uf_tiles.p, g->notuf_tiles.p, ufcnt.p);
    HIPCHK(hipGetLastError());
    int nspec = 0;
    unsigned long long ufc = 0;
    HIPCHK(hipMemcpyAsync(&nspec, fcount.p, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&ufc, ufcnt.p, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    g->sym_diff.reset(); g->sym_ho.reset(); g->sym_fused = false;   // consumed
    g->uf_count = (int64_t)ufc;
    g->nspecial = nspec;
    if (nspec == 0) { g->symmetric = 1; return DMX_OK; }
    if (nspec > kSpecLimit) { g->symmetric = 0; return DMX_OK; }
    std::vector<int32_t> specs((size_t)nspec);
    HIPCHK(copy_sync(g->ctx->stream, specs.data(), flist.p, nspec * 4, hipMemcpyDeviceToHost));
    std::sort(specs.begin(), specs.end());
    g->special_nodes = specs;
    std::vector<uint8_t> is_spec((size_t)N, 0);
    std::vector<int32_t> sidx((size_t)N, -1);
    for (int i = 0; i < nspec; i++) { is_spec[specs[i]] = 1; sidx[specs[i]] = i; }
    DevBuf<uint8_t> d_is;
    DevBuf<int32_t> d_specs, d_out;
    DevBuf<int> d_outn;
    HIPCHK(d_is.alloc(N));
    HIPCHK(d_specs.alloc(nspec));
    HIPCHK(d_out.alloc((size_t)nspec * nspec));
    HIPCHK(d_outn.alloc(nspec));
    HIPCHK(copy_sync(g->ctx->stream, d_is.p, is_spec.data(), N, hipMemcpyHostToDevice));
    HIPCHK(copy_sync(g->ctx->stream, d_specs.p, specs.data(), nspec * 4, hipMemcpyHostToDevice));
    // on the context stream: a null-stream hipMemset is not ordered before the kernel on this
    // non-blocking stream, and under load the kernel then counted from stale memory (the 4-rank
    // one-GPU rehearsal's heap abort)
    HIPCHK(hipMemsetAsync(d_outn.p, 0, nspec * 4, s));
    hipLaunchKernelGGL(sym_special_out_kernel, dim3(nspec), dim3(256), 0, s, rows, d_specs.p, nspec,
                       g->pm->d_node_cell.p, g->pm->d_cell_node.p, d_is.p, g->node_run_start.p, g->node_nruns.p,
                       g->pool.p, d_out.p, d_outn.p, nspec);
    HIPCHK(hipGetLastError());
    std::vector<int32_t> outn((size_t)nspec), out((size_t)nspec * nspec);
    HIPCHK(hipMemcpyAsync(outn.data(), d_outn.p, nspec * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(out.data(), d_out.p, (size_t)nspec * nspec * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    // A[a][b] = b in cells(a), over special nodes (asymmetric pairs only involve special nodes)
    std::vector<std::vector<char>> A((size_t)nspec, std::vector<char>((size_t)nspec, 0));
    for (int a = 0; a < nspec; a++) {
        if (outn[a] < 0) return fail(DMX_ERR_STATE, "internal: special-node list count out of range");
        for (int j = 0; j < std::min(outn[a], nspec); j++) {
            const int32_t v = out[(size_t)a * nspec + j];
            if (v < 0 || v >= N || sidx[v] < 0) return fail(DMX_ERR_STATE, "internal: special-node list entry out of range");
            A[a][sidx[v]] = 1;
        }
    }
    std::vector<std::vector<int32_t>> extra((size_t)nspec), missing((size_t)nspec);
    for (int a = 0; a < nspec; a++)
        for (int b = 0; b < nspec; b++)
            if (A[a][b] && !A[b][a]) {          // b in cells(a), a not in cells(b)
                extra[b].push_back(specs[a]);   // a is an in-neighbour of b outside cells(b)
                missing[a].push_back(specs[b]); // b sits in cells(a) but is not an in-neighbour of a
            }
    std::vector<int32_t> eoff(1, 0), moff(1, 0), ev, mv;
    for (int i = 0; i < nspec; i++) {
        ev.insert(ev.end(), extra[i].begin(), extra[i].end());
        mv.insert(mv.end(), missing[i].begin(), missing[i].end());
        eoff.push_back((int32_t)ev.size());
        moff.push_back((int32_t)mv.size());
    }
    HIPCHK(g->spec_index.alloc(N));
    HIPCHK(g->extra_off.alloc(eoff.size()));
    HIPCHK(g->missing_off.alloc(moff.size()));
    HIPCHK(g->extra.alloc(std::max<size_t>(ev.size(), 1)));
    HIPCHK(g->missing.alloc(std::max<size_t>(mv.size(), 1)));
    HIPCHK(copy_sync(g->ctx->stream, g->spec_index.p, sidx.data(), N * 4, hipMemcpyHostToDevice));
    HIPCHK(copy_sync(g->ctx->stream, g->extra_off.p, eoff.data(), eoff.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(copy_sync(g->ctx->stream, g->missing_off.p, moff.data(), moff.size() * 4, hipMemcpyHostToDevice));
    if (!ev.empty()) HIPCHK(copy_sync(g->ctx->stream, g->extra.p, ev.data(), ev.size() * 4, hipMemcpyHostToDevice));
    if (!mv.empty()) HIPCHK(copy_sync(g->ctx->stream, g->missing.p, mv.data(), mv.size() * 4, hipMemcpyHostToDevice));
    g->symmetric = 1;
    return DMX_OK;
}

// Partial-tile masks for phase C's exact test (vga_tile.hip pmask_hit): counts from the full rows
// (every rank after the rows' all-reduce), an exclusive scan into per-cell offsets, then the masks of every
// node.  Each rank builds all of them itself, with no collective: the pass costs ~0.07 s at 1000^2, where
// all-reducing its ~10 GB over the ranks would cost more, and whether a rank has them does not change
// its results (phase C scans runs without them), so the ranks need not agree.  Skipped when they would
// take more than a quarter of the free memory.
static int prepare_pmask(dmx_graph* g, int rows, int tw, int th, int tvw, int64_t Ct, bool wide) {
    dmx_ctx* ctx = g->ctx;
    hipStream_t s = ctx->stream;
    DevBuf<int64_t> cnt, scratch;
    HIPCHK(cnt.alloc(Ct));
    HIPCHK(g->poff.alloc(Ct + 1));
    HIPCHK(g->ppre.alloc((size_t)Ct * tvw));
    HIPCHK(scratch.alloc(scan_scratch_size(Ct)));
    hipLaunchKernelGGL(tile_pcount_kernel, dim3((unsigned)((Ct + 3) / 4)), dim3(256), 0, s, Ct, tvw, g->tvis.p, g->ftvis.p,
                       cnt.p, g->ppre.p);
    HIPCHK(hipGetLastError());
    scan_excl(s, cnt.p, Ct, g->poff.p, scratch.p);
    HIPCHK(hipGetLastError());
    int64_t total = 0;
    HIPCHK(copy_sync(s, &total, g->poff.p + Ct, 8, hipMemcpyDeviceToHost));
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    const size_t mask_b = (size_t)total * 8;
    bool build = total > 0 && mask_b <= free_b / 4;
    const int pmcap = wide ? PM_CAP_WIDE : PM_CAP;
    if (wide && total > 0 && tile_pmask_lds(tvw, pmcap) <= 150 * 1024) {
        // Above 1024 cells a side the masks (~80 GB at 2000^2) fit only in the scan order's place: the runs
        // are then scanned in pool order (the heads and tile-common runs stay, built from the scan order;
        // only special nodes still scan, from the first run; every regular cell phase C sees takes the masks)
        const size_t reserve = 16ull << 30;   // the search's per-workgroup buffers
        const size_t free_all = free_b + cached_bytes();
        const size_t scan_b = g->scan_pool.p ? g->scan_pool.n * sizeof(Run) + (size_t)g->nnodes * 8 +
                                                   (size_t)g->cell_scan_start.n * 12 : 0;
        if (mask_b + reserve <= free_all) {
            build = true;
        } else if (g->scan_pool.p && mask_b + reserve <= free_all + scan_b) {
            g->scan_pool.reset(); g->scan_start.reset(); g->cell_scan_start.reset(); g->cell_nruns.reset();
            g->scan_released = true;
            hipLaunchKernelGGL(tile_pool_order_kernel, dim3((unsigned)((g->nnodes + 255) / 256)), dim3(256), 0, s, rows, tw,
                               g->pm->d_node_cell.p, g->nnodes, g->node_run_start.p, g->tscan_start.p);
            HIPCHK(hipGetLastError());
            VLOG("vga prep: scan order released for %.1f GB of partial-tile masks\n", mask_b / 1e9);
            build = true;
            if (getenv("DMX_VGA_PMASK_FAIL"))   // test hook: a failure after the release (the next call recovers)
                return fail(DMX_ERR_HIP, "injected failure after the scan order was released");
        } else {
            build = false;
        }
    }
    if (!build) {
        g->poff.reset();
        g->ppre.reset();
        return DMX_OK;
    }
    HIPCHK(g->pmask.alloc((size_t)total));
    HIPCHK(hipMemsetAsync(g->pmask.p, 0, mask_b, s));
    const int64_t N = g->nnodes;
    if (N > 0) {
        const int64_t nb = std::min<int64_t>(N, (int64_t)ctx->num_cu * 16);
        hipLaunchKernelGGL(tile_pmask_kernel, dim3((unsigned)nb), dim3(64 * TV_WAVES), tile_pmask_lds(tvw, pmcap), s, rows,
                           tw, th, g->pm->d_node_cell.p, N, g->node_run_start.p, g->node_nruns.p, g->pool.p, g->tvis.p,
                           g->ftvis.p, g->poff.p, g->pmask.p, pmcap);
        HIPCHK(hipGetLastError());
    }
    return DMX_OK;
}

// Which memory-dependent VGA preparation structures the graph holds (last_stats[40..42]; bench.py prints them):
// the search a call takes depends on what fitted next to the graph (DESIGN.md sections 1 and 5).
static void prep_state_stats(dmx_ctx* ctx, const dmx_graph* g) {
    long long f = 0;
    if (g->scan_pool.p) f |= 1;          // the BFS scan order
    if (g->scan_released) f |= 2;        // ... released for the masks (runs read in pool order)
    if (g->tvis.p) f |= 4;               // tile-visibility rows
    if (g->ftvis.p) f |= 8;              // fully-seen tile rows
    if (g->ttvis.p) f |= 16;             // tile-to-tile rows
    if (g->pmask.p) f |= 32;             // partial-tile masks
    if (g->tvsum.p || g->tvnz.p) f |= 64;   // row summaries
    ctx->last_stats[40] = f;
    ctx->last_stats[41] = (long long)((g->tvis.p ? g->tvis.n * 8 : 0) + (g->ftvis.p ? g->ftvis.n * 8 : 0) +
                                      (g->ttvis.p ? g->ttvis.n * 8 : 0) + (g->tvsum.p ? g->tvsum.n * 8 : 0) + (g->tvnz.p ? g->tvnz.n * 8 : 0));
    ctx->last_stats[42] = (long long)(g->scan_pool.p ? g->scan_pool.n * sizeof(Run) : 0);
}

// LDS of the tile BFS workgroup: the frontier bitmap (unless FG), the tile-row summary Fsr, then either the
// per-tile column summary Fsc or the line-resolved summaries RB / CB, then the level histogram.  Returns the
// bytes (0: does not fit) and the variant: *fg the frontier in HBM, *rbm the line summaries.
static size_t tile_lds_layout(int tw, int th, bool* fg, bool* rbm) {
    const size_t nt = (size_t)tw * th, wr_ = (tw + 63) / 64, wc_ = (th + 63) / 64;
    const size_t lds_f = nt * 8, lds_h = (size_t)VGA_HMAX * 4;
    const size_t lds_sc = (size_t)(th * wr_ + tw * wc_) * 8, lds_rbcb = (size_t)(th * wr_ + th * 8 * wr_ + tw * 8 * wc_) * 8;
    const size_t lds_cap = (size_t)160 * 1024 - 1024;
    const char* rb_env = getenv("DMX_VGA_RB");
    const bool rb_ok = !(rb_env && atoi(rb_env) == 0);
    *fg = false;
    *rbm = false;
    if (rb_ok && lds_f + lds_rbcb + lds_h <= lds_cap) { *rbm = true; return lds_f + lds_rbcb + lds_h; }
    if (lds_f + lds_sc + lds_h <= lds_cap) return lds_f + lds_sc + lds_h;
    if (rb_ok && lds_rbcb + lds_h <= lds_cap) { *fg = true; *rbm = true; return lds_rbcb + lds_h; }
    if (lds_sc + lds_h <= lds_cap) { *fg = true; return lds_sc + lds_h; }
    return 0;
}

// Tile-ordered per-cell arrays, head runs and tile-common runs for vga_tile_kernel (O(runs)).
static int prepare_tiles(dmx_graph* g) {
    if (g->tiles_ready) return DMX_OK;
    // a preparation that released the scan order for the masks and then failed (prepare_pmask) left the tile data
    // half built: rebuild the scan order before the heads and the tile-common runs read it
    if (g->scan_released)
        if (int rc = restore_scan_order(g)) return rc;
    dmx_ctx* ctx = g->ctx;
    hipStream_t s = ctx->stream;
    PointMapHost& h = *g->pm->host;
    const int cols = h.cols(), rows = h.rows();
    const int tw = (cols + 7) / 8, th = (rows + 7) / 8, nt = tw * th;
    const int64_t N = g->nnodes, Ct = (int64_t)nt * 64;
    HIPCHK(g->tscan_start.alloc(Ct));
    HIPCHK(g->tnruns.alloc(Ct));
    HIPCHK(g->heads.alloc((size_t)KH * Ct));
    HIPCHK(g->cr.alloc((size_t)CRK * nt));
    HIPCHK(g->regular_tiles.alloc(nt));
    HIPCHK(hipMemsetAsync(g->tnruns.p, 0, Ct * 4, s));
    HIPCHK(hipMemsetAsync(g->tscan_start.p, 0, Ct * 8, s));
    HIPCHK(hipMemsetAsync(g->heads.p, 0xFF, (size_t)KH * Ct * sizeof(Run), s));
    // regular = U_f minus the special (asymmetric) nodes
    std::vector<unsigned long long> uf((size_t)nt);
    HIPCHK(hipMemcpyAsync(uf.data(), g->uf_tiles.p, nt * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (int32_t k : g->special_nodes) {
        const int c = g->pm->node_cell[k];
        const int x = c / rows, y = c % rows;
        uf[(size_t)(y >> 3) * tw + (x >> 3)] &= ~(1ull << ((y & 7) * 8 + (x & 7)));
    }
    HIPCHK(hipMemcpyAsync(g->regular_tiles.p, uf.data(), nt * 8, hipMemcpyHostToDevice, s));
    if (N) {
        hipLaunchKernelGGL(tile_heads_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, rows, tw,
                           g->pm->d_node_cell.p, N, g->node_nruns.p, g->scan_pool.p, g->scan_start.p,
                           g->tscan_start.p, g->tnruns.p, g->heads.p, (size_t)Ct);
        HIPCHK(hipGetLastError());
    }
    const int dmax = std::max(cols, rows);
    const size_t lds = (size_t)8 * (dmax + 2) * 4;
    // a capacity of the tile path: the callers fall back to the direction-optimising / top-down searches
    if (lds > 150 * 1024) return fail(DMX_ERR_CAPACITY, "grid too long for the tile-common-run pass");
    hipLaunchKernelGGL(tile_cr_kernel, dim3((unsigned)std::min<int64_t>(nt, (int64_t)ctx->num_cu * 8)), dim3(CR_THREADS),
                       lds, s, cols, rows, tw, th, g->regular_tiles.p, g->pm->d_cell_node.p, g->node_run_start.p,
                       g->node_nruns.p, g->scan_start.p, g->scan_pool.p, g->pool.p, dmax, g->cr.p);
    HIPCHK(hipGetLastError());
    // tile-visibility rows (phase C rejects cells with no frontier tile in view); ~2 KB per cell at
    // 1000^2, skipped when they would not fit comfortably
    const int tvw = th * ((tw + 63) / 64);
    const size_t tv_bytes = (size_t)Ct * tvw * 8;
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    const char* tv_env = getenv("DMX_VGA_TVIS");
    const bool tv_on = !(tv_env && atoi(tv_env) == 0);
    const char* ftv_env = getenv("DMX_VGA_FTVIS");
    const bool ftv_on = !(ftv_env && atoi(ftv_env) == 0);
    // Grids up to 1024 cells a side (tvw <= 256: the masks' row test reads 4 words a lane): tvis, ftvis, the
    // tile rows and the partial-tile masks when they take at most a quarter of the free memory.  Wider grids
    // (2000^2: 8 KB a row, 32 GB) keep tvis, the phase-C miss certificate in front of the run scan, when it takes
    // at most a third of what is free next to the graph and its scan order, and ftvis too (the certain-hit
    // test) when both leave 24 GiB free for the search's own buffers.
    const bool wide = tvw > 256;
    const size_t free_all = free_b + cached_bytes();
    // (the wide-grid ftvis, tile rows and masks serve the HBM-frontier variant, whose code reads wide rows; a
    // wide grid whose frontier fits the LDS -- a few tiles high, very long -- keeps tvis alone)
    bool fg_grid = false, rbm_grid = false;
    tile_lds_layout(tw, th, &fg_grid, &rbm_grid);
    bool ftv = ftv_on && (!wide || (fg_grid && 2 * tv_bytes + (24ull << 30) <= free_all));
    bool tv_build = tv_on && N && tv_bytes <= (32ull << 30) &&
                    (wide ? tv_bytes <= free_all / 3 : tv_bytes * (ftv ? 2 : 1) <= free_b / 4);
    if (g->prep_fn) {
        // every rank must take the same branches (the rows are all-reduced): build only what all can
        DevBuf<int64_t> veto;
        HIPCHK(veto.alloc(1));
        const int64_t v = (tv_build ? 0 : 1) + (ftv ? 0 : (1ll << 20));
        HIPCHK(hipMemcpyAsync(veto.p, &v, 8, hipMemcpyHostToDevice, s));
        if (int rc = prep_allreduce(g, veto.p, 1, DMX_I64)) return rc;
        int64_t vs = 0;
        HIPCHK(copy_sync(g->ctx->stream, &vs, veto.p, 8, hipMemcpyDeviceToHost));
        tv_build = (vs & ((1ll << 20) - 1)) == 0;
        ftv = (vs >> 20) == 0;
    }
    if (tv_build) {
        HIPCHK(g->tvis.alloc(Ct * tvw));
        HIPCHK(hipMemsetAsync(g->tvis.p, 0, tv_bytes, s));
        if (ftv) {
            HIPCHK(g->ftvis.alloc(Ct * tvw));
            HIPCHK(hipMemsetAsync(g->ftvis.p, 0, tv_bytes, s));
        }
        const int ncw = (nt + 3) / 4;
        const size_t tv_lds = ((size_t)(ncw + 1) / 2 + (size_t)(tvw + (ncw + 1) / 2)) * 8;   // one node per workgroup
        if (tv_lds > 150 * 1024) return fail(DMX_ERR_CAPACITY, "grid too large for the tile-visibility pass");
        int64_t pb, pe;
        prep_range(g, pb, pe);
        if (pe > pb) {
            const int64_t nb = std::min<int64_t>(pe - pb, (int64_t)ctx->num_cu * 16);
            hipLaunchKernelGGL(tile_vis_kernel, dim3((unsigned)nb), dim3(64 * TV_WAVES), tv_lds, s, rows, tw, th,
                               g->pm->d_node_cell.p + pb, pe - pb, g->node_run_start.p + pb, g->node_nruns.p + pb,
                               g->pool.p, g->notuf_tiles.p, g->tvis.p, ftv ? g->ftvis.p : nullptr);
            HIPCHK(hipGetLastError());
        }
        // rows of distinct nodes are disjoint: the sum over ranks is their union
        if (int rc = prep_allreduce(g, g->tvis.p, Ct * tvw, DMX_I64)) return rc;
        if (ftv)
            if (int rc = prep_allreduce(g, g->ftvis.p, Ct * tvw, DMX_I64)) return rc;
        const char* tt_env = getenv("DMX_VGA_TTVIS");
        if (ftv && !(tt_env && atoi(tt_env) == 0)) {
            HIPCHK(g->ttvis.alloc((size_t)2 * nt * tvw));   // ttvis, then ttany
            hipLaunchKernelGGL(tile_tt_kernel, dim3((unsigned)((nt + 3) / 4)), dim3(256), 0, s, nt, tvw, g->regular_tiles.p,
                               g->ftvis.p, g->tvis.p, g->ttvis.p, g->ttvis.p + (size_t)nt * tvw);
            HIPCHK(hipGetLastError());
        }
        const char* pm_env = getenv("DMX_VGA_PMASK");
        // (wide grids: the masks need the row summaries, at most 64 words of them, and a 16-bit row prefix)
        if (ftv && !(pm_env && atoi(pm_env) == 0) && (!wide || ((tvw + 63) / 64 <= 64 && nt <= 65535)))
            if (int rc = prepare_pmask(g, rows, tw, th, tvw, Ct, wide)) return rc;
        // the row summaries keep word k in lane k (vga_tile.hip reads them with readlane): at most 64 words
        if (wide && (tvw + 63) / 64 <= 64) {
            HIPCHK(g->tvsum.alloc((size_t)Ct * ((tvw + 63) / 64)));
            hipLaunchKernelGGL(tile_vsum_kernel, dim3((unsigned)((Ct + 3) / 4)), dim3(256), 0, s, Ct, tvw, g->tvis.p,
                               g->tvsum.p);
            HIPCHK(hipGetLastError());
        }
        // narrow grids with the masks: phase C's row loads skip the cell's zero words (1000^2: 61 % of the words
        // under a frontier tile row are zero; 32 B a cell)
        const char* nz_env = getenv("DMX_VGA_TVNZ");
        if (VGA_TVNZ && !wide && ftv && g->pmask.p && !(nz_env && atoi(nz_env) == 0)) {
            HIPCHK(g->tvnz.alloc((size_t)Ct * ((tvw + 63) / 64)));
            hipLaunchKernelGGL(tile_vsum_kernel, dim3((unsigned)((Ct + 3) / 4)), dim3(256), 0, s, Ct, tvw, g->tvis.p,
                               g->tvnz.p);
            HIPCHK(hipGetLastError());
        }
        g->tvw = tvw;
    }
    HIPCHK(hipStreamSynchronize(s));
    g->tiles_ready = true;
    return DMX_OK;
}

// threads of the tile BFS workgroup on grids above 4096 tiles (one workgroup per CU either way: F takes the
// LDS); A/B builds: -DVGA_NT_BIG=512
#ifndef VGA_NT_BIG
#define VGA_NT_BIG 1024
#endif
// The reference's own level order (vga_ordered.hip) for the searches the level-synchronous kernels cannot
// answer (merge links with a context-filled odd end found together with the other end at one level).
// VGA global: one search per listed source node, its level histogram into the measures kernel (rows of `outp`,
// levels into d_levels).  Visual step depth (seed_cells non-empty, PixelRef order): one search, the level of
// every cell it reaches into d_cell_level [C].
static int ordered_search(dmx_ctx* ctx, dmx_graph* g, double radius, const std::vector<int32_t>& src,
                          const std::vector<int32_t>& seed_cells, float* outp, int64_t* d_levels, int32_t* d_cell_level) {
    const PointMapHost& h = *g->pm->host;
    const int64_t C = h.cells(), N = g->nnodes;
    const bool vsd = !seed_cells.empty();
    const int64_t nsearch = vsd ? 1 : (int64_t)src.size();
    if (nsearch == 0) return DMX_OK;
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    const size_t per = (size_t)C * 5 + (size_t)N * 8;   // misc, extents, two level vectors
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>({nsearch, (int64_t)ctx->num_cu,
                                                                    (int64_t)((free_b + cached_bytes()) / 4 / per)}));
    DevBuf<uint8_t> misc;
    DevBuf<int16_t> ext;
    DevBuf<int32_t> vec, d_src, d_seeds, hist, nlev;
    DevBuf<unsigned long long> junk;
    HIPCHK(misc.alloc((size_t)blocks * C));
    HIPCHK(ext.alloc((size_t)blocks * 2 * C));
    HIPCHK(vec.alloc((size_t)blocks * 2 * std::max<int64_t>(N, 1)));
    OrderedParams P;
    P.rows = h.rows(); P.C = C; P.N = N;
    P.node_run_start = g->node_run_start.p; P.node_nruns = g->node_nruns.p; P.pool = g->pool.p;
    P.cell_node = g->pm->d_cell_node.p; P.node_cell = g->pm->d_node_cell.p; P.node_flags = g->pm->d_node_flags.p;
    P.merge_cell = g->merges.empty() ? nullptr : g->d_merge_cell.p;
    P.src = nullptr; P.nsrc = 0; P.radius = (int)radius; P.hist_all = nullptr; P.nlev_all = nullptr;
    // levels kept per search: a radius r search has at most r + 2 (the cells at level r are counted, not
    // expanded); radius n as deep as the direction-optimising kernel follows (vga_do: 4096 levels)
    P.hmax = (radius == -1.0) ? 4096 : (int)std::min<double>(4096.0, radius + 2.0);
    P.seeds = nullptr; P.nseeds = 0; P.cell_level = d_cell_level;
    P.misc = misc.p; P.ext = ext.p; P.vec = vec.p;
    P.error = ctx->counters.p + 1;
    P.work_counter = ctx->counters.p + 0;
    P.ctl = ctx->d_ctl;
    ctx->h_ctl->progress = 0;
    HIPCHK(hipMemsetAsync(ctx->counters.p, 0, 2 * sizeof(int), ctx->stream));
    if (vsd) {
        HIPCHK(d_seeds.alloc(seed_cells.size()));
        HIPCHK(hipMemcpyAsync(d_seeds.p, seed_cells.data(), seed_cells.size() * 4, hipMemcpyHostToDevice, ctx->stream));
        P.seeds = d_seeds.p; P.nseeds = (int)seed_cells.size();
    } else {
        HIPCHK(d_src.alloc(src.size()));
        HIPCHK(hist.alloc((size_t)nsearch * P.hmax));
        HIPCHK(nlev.alloc(nsearch));
        HIPCHK(hipMemcpyAsync(d_src.p, src.data(), src.size() * 4, hipMemcpyHostToDevice, ctx->stream));
        P.src = d_src.p; P.nsrc = (int)src.size(); P.hist_all = hist.p; P.nlev_all = nlev.p;
    }
    DevBuf<OrderedParams> dP;
    HIPCHK(dP.alloc(1));
    HIPCHK(hipMemcpyAsync(dP.p, &P, sizeof(P), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(vga_ordered_kernel, dim3((unsigned)blocks), dim3(ORD_NT), 0, ctx->stream, (const OrderedParams*)dP.p);
    HIPCHK(hipGetLastError());
    HIPCHK(wait_progress(ctx, DMX_PHASE_VGA, nsearch, 1));   // progress posts, the cancel flag
    CANCEL_POINT(ctx);
    int err = 0;
    HIPCHK(copy_sync(ctx->stream, &err, ctx->counters.p + 1, sizeof(int), hipMemcpyDeviceToHost));
    // deeper than the reference-order search keeps (the engine's own deepest search): declined, so that a
    // caller with a CPU path (integration/dmx_salalib.cpp) can take it
    if (err) return fail(DMX_ERR_UNSUPPORTED, "VGA BFS in the reference's order deeper than 4096 levels");
    if (!vsd) {
        HIPCHK(junk.alloc(32));
        hipLaunchKernelGGL(vga_measures_kernel, dim3((unsigned)((nsearch + 255) / 256)), dim3(256), 0, ctx->stream,
                           (int64_t)0, nsearch, hist.p, nlev.p, outp, d_levels, junk.p, (const int32_t*)d_src.p, P.hmax, true);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
    VLOG("reference-order searches: %lld on %lld workgroups\n", (long long)nsearch, (long long)blocks);
    return DMX_OK;
}

// The sources a level-synchronous kernel marked in d_oflag, run again in the reference's order.
static int vga_order_rerun(dmx_ctx* ctx, dmx_graph* g, double radius, const uint8_t* d_oflag, float* outp,
                           int64_t* d_levels) {
    const int64_t N = g->nnodes;
    std::vector<uint8_t> fl((size_t)N);
    HIPCHK(copy_sync(ctx->stream, fl.data(), d_oflag, (size_t)N, hipMemcpyDeviceToHost));
    std::vector<int32_t> src;
    for (int64_t k = 0; k < N; k++)
        if (fl[k]) src.push_back((int32_t)k);
    const double t0 = now_s();
    int rc = ordered_search(ctx, g, radius, src, {}, outp, d_levels, nullptr);
    ctx->last_vga_s += now_s() - t0;
    ctx->last_stats[38] = (int64_t)src.size();
    return rc;
}

extern "C++" template <int NT, bool SPECIAL, bool RBM, bool FG>
static int launch_tile(dmx_ctx* ctx, const VgaTileParams& Q, int64_t nsrc, size_t lds, int64_t* blocks_out,
                       DevBuf<unsigned long long>& xg, DevBuf<int4>& queue, DevBuf<int32_t>& list) {
    // The shapes the kernel and its grid assume, checked before the launch: a tile grid that covers
    // the cells, the frontier (FG false) and the summaries inside the dynamic LDS, row words the fused phase-C
    // test covers (4 a lane: 256), the 32-bit narrow hint's tile (15 bits) and mask slot (16 bits; a cell's
    // partial tiles are at most nt), the asymmetric-mode list capacity.
    {
        const int64_t nt = (int64_t)Q.tw * Q.th;
        const char* why = nullptr;
        if (Q.tw != (Q.cols + 7) / 8 || Q.th != (Q.rows + 7) / 8 || nt <= 0) why = "tile grid does not cover the cells";
        else if (lds > (size_t)160 * 1024) why = "dynamic LDS above 160 KiB";
        else if (!FG && (size_t)nt * 8 > lds) why = "frontier bitmap larger than the dynamic LDS";
        else if (Q.tvis && Q.tvw != Q.th * ((Q.tw + 63) / 64)) why = "tile-visibility row width differs from the tile grid";
        else if (!FG && Q.pmask && Q.tvw > 256) why = "row words past the fused phase-C test (256)";
        else if (Q.tvnz && (FG || Q.tvw > 256)) why = "narrow row summaries on a wide grid";
        else if (Q.pmask && !FG && nt > 32767) why = "narrow mask hint: tile index above 15 bits";
        else if (Q.asym_tiles && Q.alist_cap <= 0) why = "asymmetric mode without an A-cell list";
        if (why) return fail(DMX_ERR_STATE, (std::string("VGA tile launch: ") + why).c_str());
    }
    int occ = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, vga_tile_kernel<NT, SPECIAL, RBM, FG>, NT, lds));
    if (occ < 1) occ = 1;
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((int64_t)ctx->num_cu * occ, nsrc));
    const int64_t nt = (int64_t)Q.tw * Q.th;
    HIPCHK(xg.alloc((size_t)blocks * (FG ? 3 : 2) * nt));   // V, X [, F]
    HIPCHK(queue.alloc((size_t)blocks * nt));
    HIPCHK(list.alloc((size_t)blocks * nt * 64 * 2));
    DevBuf<int32_t> tlist;   // per workgroup: the two unvisited-tile lists
    HIPCHK(tlist.alloc((size_t)blocks * nt * 2));
    DevBuf<uint32_t> hint;
    HIPCHK(hint.alloc((size_t)nt * 64));
    HIPCHK(hipMemsetAsync(hint.p, 0xFF, (size_t)nt * 64 * 4, ctx->stream));
    DevBuf<uint32_t> hint2;   // (narrow grids with the masks) the second, fully-seen-tile hint
    DevBuf<int32_t> mseen;   // per workgroup: merge_order_check stamps
    DevBuf<int32_t> alist;   // asymmetric mode: per workgroup, the frontier's A cells
    VgaTileParams P = Q;
    P.hint2 = nullptr;
    if (VGA_H2 > 0 && Q.pmask && !FG && !getenv("DMX_VGA_NOHINT2")) {
        HIPCHK(hint2.alloc((size_t)nt * 64 * VGA_H2));
        HIPCHK(hipMemsetAsync(hint2.p, 0xFF, (size_t)nt * 64 * 4 * VGA_H2, ctx->stream));
        P.hint2 = hint2.p;
    }
    if (Q.asym_tiles) {
        HIPCHK(alist.alloc((size_t)blocks * Q.alist_cap));
        P.alist = alist.p;
    }
    P.fg = FG ? xg.p + (size_t)blocks * 2 * nt : nullptr;   // per workgroup [nt] after every V / X pair
    if (Q.nmamb) {
        HIPCHK(mseen.alloc((size_t)blocks * Q.nmamb));
        HIPCHK(hipMemsetAsync(mseen.p, 0, (size_t)blocks * Q.nmamb * 4, ctx->stream));
        P.mseen = mseen.p;
    }
    P.xg = xg.p;
    P.queue = queue.p;
    P.list = list.p;
    P.tlist = tlist.p;
    P.hint = hint.p;
    DevBuf<unsigned long long> hintw;   // (wide grids with the masks) mask hints
    P.hintw = nullptr;
    if (P.pmask && P.tvsum) {
        HIPCHK(hintw.alloc((size_t)nt * 64));
        HIPCHK(hipMemsetAsync(hintw.p, 0, (size_t)nt * 64 * 8, ctx->stream));
        P.hintw = hintw.p;
    }
    // chunks of consecutive sources per workgroup, small enough to balance the tail
    P.chunk = 1;   // concurrent workgroups on neighbouring sources share L2 lines and hints
    if (const char* c = getenv("DMX_VGA_CHUNK")) P.chunk = std::max(1, atoi(c));
    P.nwork = (int)((P.src_end - P.src_begin + P.chunk - 1) / P.chunk);
    HIPCHK(hipEventRecord(ctx->ev0, ctx->stream));
    P.ctl = ctx->d_ctl;
    ctx->h_ctl->progress = 0;
    DevBuf<VgaTileParams> dP;
    HIPCHK(dP.alloc(1));
    HIPCHK(hipMemcpyAsync(dP.p, &P, sizeof(P), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL((vga_tile_kernel<NT, SPECIAL, RBM, FG>), dim3((unsigned)blocks), dim3(NT), lds, ctx->stream,
                       (const VgaTileParams*)dP.p);
    HIPCHK(hipGetLastError());
    HIPCHK(wait_progress(ctx, DMX_PHASE_VGA, nsrc, P.chunk));   // hint freed on return
    *blocks_out = blocks;
    return DMX_OK;
}

static int vga_tile_impl(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t sb, int64_t se, float* out,
                         bool out_on_device, int64_t* levels, int tw, int th, const int32_t* d_seeds = nullptr,
                         int nseeds = 0, int32_t* d_cell_level = nullptr, const int32_t* d_src_list = nullptr,
                         dmx_graph* pg = nullptr) {
    // pg (asymmetric mode): the graph analysed; g is its symmetric reference (prepare_asym)
    int rc = prepare_tiles(g);
    if (rc) return rc;
    PointMapHost& h = *g->pm->host;
    const int64_t N = g->nnodes, nsrc = se - sb;
    const int nt = tw * th;
    const int maxlev = 1024;
    DevBuf<float> d_out;
    float* outp = out;
    if (!out_on_device) {
        HIPCHK(d_out.alloc(std::max<int64_t>(N, 1) * 7));
        outp = d_out.p;
    }
    DevBuf<int64_t> d_lv;
    if (levels) HIPCHK(d_lv.alloc(std::max<int64_t>(N, 1) * 3));
    HIPCHK(hipMemsetAsync(ctx->counters.p, 0, 16 * sizeof(int), ctx->stream));
    HIPCHK(hipMemsetAsync(ctx->stats.p, 0, 32 * sizeof(unsigned long long), ctx->stream));
    VgaTileParams Q;
    Q.cols = h.cols(); Q.rows = h.rows(); Q.tw = tw; Q.th = th;
    Q.seed_tiles = g->notuf_tiles.p; Q.regular_tiles = g->regular_tiles.p; Q.nonexp_tiles = g->pm->d_nonexp_tiles.p;
    Q.cr = g->cr.p; Q.heads = g->heads.p; Q.tscan_start = g->tscan_start.p; Q.tnruns = g->tnruns.p;
    Q.scan_pool = g->scan_released ? g->pool.p : g->scan_pool.p;   // (tscan_start then indexes the pool)
    Q.tvis = g->tvw ? g->tvis.p : nullptr; Q.tvw = g->tvw;
    Q.tvsum = (g->tvw && g->tvsum.p) ? g->tvsum.p : nullptr;
    Q.tvnz = (g->tvw && g->tvnz.p) ? g->tvnz.p : nullptr;
    Q.ftvis = (g->tvw && g->ftvis.p) ? g->ftvis.p : nullptr;
    Q.ttvis = (g->tvw && g->ttvis.p) ? g->ttvis.p : nullptr;
    Q.ttany = Q.ttvis ? g->ttvis.p + (size_t)tw * th * g->tvw : nullptr;
    const char* pmk_env = getenv("DMX_VGA_PMASK");   // also a launch-time switch (the masks stay built), except
    // where the masks replaced the scan order (phase C's scan of the regular cells reads the scan order)
    Q.pmask = (Q.ftvis && g->pmask.p && (g->scan_released || !(pmk_env && atoi(pmk_env) == 0))) ? g->pmask.p : nullptr;
    Q.poff = Q.pmask ? g->poff.p : nullptr;
    Q.ppre = Q.pmask ? g->ppre.p : nullptr;
    Q.node_cell = g->pm->d_node_cell.p; Q.cell_node = g->pm->d_cell_node.p; Q.node_flags = g->pm->d_node_flags.p;
    Q.node_run_start = g->node_run_start.p; Q.node_nruns = g->node_nruns.p; Q.pool = g->pool.p;
    const bool corr = g->nspecial > 0;
    Q.spec_index = corr ? g->spec_index.p : nullptr;
    Q.extra_off = corr ? g->extra_off.p : nullptr;
    Q.extra = corr ? g->extra.p : nullptr;
    Q.missing_off = corr ? g->missing_off.p : nullptr;
    Q.missing = corr ? g->missing.p : nullptr;
    Q.src_begin = sb; Q.src_end = se; Q.radius = (int)radius; Q.gates_only = gates_only;
    Q.uf_count = g->uf_count;
    Q.seeds = d_seeds; Q.nseeds = nseeds; Q.cell_level = d_cell_level;
    Q.nmp = (int)(g->merges.size() / 2);
    Q.mpairs = Q.nmp ? g->d_mpairs.p : nullptr;
    Q.nmamb = Q.nmp && radius != -1.0 ? g->nmamb : 0;
    Q.mamb = Q.nmamb ? g->d_mamb.p : nullptr;
    Q.mseen = nullptr;
    DevBuf<uint8_t> oflag;   // sources whose result depends on the reference's pop order (merge_order_check)
    Q.oflag = nullptr;
    if (Q.nmamb) {
        HIPCHK(oflag.alloc(std::max<int64_t>(N, 1)));
        HIPCHK(hipMemsetAsync(oflag.p, 0, (size_t)std::max<int64_t>(N, 1), ctx->stream));
        Q.oflag = oflag.p;
    }
    Q.src_list = d_src_list;   // [sb, se) index this list of source nodes (out must be on the device)
    Q.asym_tiles = nullptr; Q.asym_uf = nullptr; Q.apool = nullptr; Q.arun_start = nullptr; Q.anruns = nullptr;
    Q.alist = nullptr; Q.alist_cap = 0;
    if (pg) {   // asymmetric mode: pg's own universe (pre-visited cells, early-exit count) and runs for A's pushes
        Q.seed_tiles = pg->notuf_tiles.p;
        Q.uf_count = pg->uf_count;
        Q.asym_tiles = pg->asym_tiles.p;
        Q.asym_uf = g->uf_tiles.p;
        Q.apool = pg->pool.p; Q.arun_start = pg->node_run_start.p; Q.anruns = pg->node_nruns.p;
        Q.alist_cap = (int)std::max<int64_t>(pg->nasym, 1);
    }
    // Beamer's direction test on cell counts (top-down levels run on the LDS frontier bitmap)
    Q.alpha = 60;   // top-down costs a frontier cell its whole run list (~R/N runs): keep it rare
    if (const char* a = getenv("DMX_VGA_ALPHA")) Q.alpha = atoi(a);
    Q.bext = BEXT_DEFAULT;
    if (const char* b = getenv("DMX_VGA_BEXT")) Q.bext = std::max(0, atoi(b));
    Q.crk = 4;   // all 4 tile-common runs: the last two save ~20% of the phase-B cell tests
    if (const char* c = getenv("DMX_VGA_CRK")) Q.crk = std::min(CRK, std::max(0, atoi(c)));
    Q.work_counter = ctx->counters.p + 0; Q.error = ctx->counters.p + 1;
    DevBuf<int32_t> d_hist, d_nlev;
    HIPCHK(d_hist.alloc((size_t)std::max<int64_t>(N, 1) * VGA_HMAX));
    HIPCHK(d_nlev.alloc(std::max<int64_t>(N, 1)));
    Q.maxlev = maxlev; Q.hist_out = d_hist.p; Q.nlev_out = d_nlev.p; Q.stats = ctx->stats.p;
    bool fg = false, rbm = false;
    const size_t L = tile_lds_layout(tw, th, &fg, &rbm);
    if (!L) return fail(DMX_ERR_CAPACITY, "grid too large for the tile BFS's LDS summaries");
    // With the frontier in HBM a top-down level's run rasterisation takes global atomics: past level 1 the
    // bottom-up levels win (2000^2 interior block: alpha 60 -> 200: 2.70 -> 2.28 s, identical output;
    // 1000 and 100000 the same, profiles/r5_vga2000_alpha.jsonl)
    if (fg && !getenv("DMX_VGA_ALPHA")) Q.alpha = 1000;
    DevBuf<unsigned long long> xg;
    DevBuf<int4> queue;
    DevBuf<int32_t> list;
    int64_t blocks = 0;
    int kt = 0, ntpb = 0;
    (void)kt;
    if (nsrc > 0) {
        const bool sp = g->nspecial > 0;
        if (fg) {
            rc = sp ? (rbm ? launch_tile<1024, true, true, true>(ctx, Q, nsrc, L, &blocks, xg, queue, list)
                           : launch_tile<1024, true, false, true>(ctx, Q, nsrc, L, &blocks, xg, queue, list))
                    : (rbm ? launch_tile<1024, false, true, true>(ctx, Q, nsrc, L, &blocks, xg, queue, list)
                           : launch_tile<1024, false, false, true>(ctx, Q, nsrc, L, &blocks, xg, queue, list));
            ntpb = 1024;
        } else if (nt <= 4096) {
            rc = sp ? (rbm ? launch_tile<256, true, true, false>(ctx, Q, nsrc, L, &blocks, xg, queue, list)
                           : launch_tile<256, true, false, false>(ctx, Q, nsrc, L, &blocks, xg, queue, list))
                    : (rbm ? launch_tile<256, false, true, false>(ctx, Q, nsrc, L, &blocks, xg, queue, list)
                           : launch_tile<256, false, false, false>(ctx, Q, nsrc, L, &blocks, xg, queue, list));
            ntpb = 256;
        } else {
            rc = sp ? (rbm ? launch_tile<VGA_NT_BIG, true, true, false>(ctx, Q, nsrc, L, &blocks, xg, queue, list)
                           : launch_tile<VGA_NT_BIG, true, false, false>(ctx, Q, nsrc, L, &blocks, xg, queue, list))
                    : (rbm ? launch_tile<VGA_NT_BIG, false, true, false>(ctx, Q, nsrc, L, &blocks, xg, queue, list)
                           : launch_tile<VGA_NT_BIG, false, false, false>(ctx, Q, nsrc, L, &blocks, xg, queue, list));
            ntpb = VGA_NT_BIG;
        }
        if (rc) return rc;
        CANCEL_POINT(ctx);
        if (nseeds == 0) {
            hipLaunchKernelGGL(vga_measures_kernel, dim3((unsigned)((nsrc + 255) / 256)), dim3(256), 0, ctx->stream, sb,
                               se, d_hist.p, d_nlev.p, outp, levels ? d_lv.p : nullptr, ctx->stats.p, d_src_list);
            HIPCHK(hipGetLastError());
        }
        HIPCHK(hipEventRecord(ctx->ev1, ctx->stream));
    } else {
        HIPCHK(hipEventRecord(ctx->ev0, ctx->stream));
        HIPCHK(hipEventRecord(ctx->ev1, ctx->stream));
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->last_vga_s = ms * 1e-3;
    int hc[2];
    HIPCHK(copy_sync(ctx->stream, hc, ctx->counters.p, sizeof(hc), hipMemcpyDeviceToHost));
    if (hc[1] & ~KERR_ORDER) return fail(DMX_ERR_CAPACITY, "VGA BFS exceeded its level capacity");
    ctx->last_stats[38] = 0;
    if ((hc[1] & KERR_ORDER) && nseeds == 0)
        if (int rc2 = vga_order_rerun(ctx, g, radius, oflag.p, outp, levels ? d_lv.p : nullptr)) return rc2;
    unsigned long long st[32];
    HIPCHK(copy_sync(ctx->stream, st, ctx->stats.p, sizeof(st), hipMemcpyDeviceToHost));
    for (int i = 0; i < 5; i++) ctx->phase_cycles[i] = (long long)st[8 + i];
    ctx->last_stats[18] = (long long)st[16];                          // phase-C hits by a fully seen tile
    ctx->last_stats[19] = (long long)st[17];                          // clocks of top-down levels > 1
    ctx->last_stats[20] = (long long)st[18];                          // phase-B tiles
    ctx->last_stats[21] = (long long)st[19];                          // phase-B cells
    ctx->last_stats[22] = (long long)st[20];                          // phase-B tiles resolved by ttvis
    ctx->last_stats[27] = (long long)st[25];                          // phase-B tiles pruned by ttany
    ctx->last_stats[28] = (long long)st[26];                          // phase-B row-test clocks (not collected: 0)
    ctx->last_stats[29] = (long long)st[27];                          // phase-B tiles with cell tests
    ctx->last_stats[30] = (long long)st[28];                          // phase-B cell-test clocks (not collected: 0)
    ctx->last_stats[31] = (long long)st[29];                          // phase-B cells past hint + 4 heads
    ctx->last_stats[23] = (long long)st[21];                          // phase-C busy clocks summed over waves
    ctx->last_stats[24] = (long long)st[22];                          // phase-C per-cell clocks (not collected: 0)
    ctx->last_stats[25] = (long long)st[23];                          // phase-C special-node clocks (not collected: 0)
    ctx->last_stats[26] = (long long)st[24];                          // phase-C special-node tests
    ctx->last_stats[3] = 3 | ((long long)g->nspecial << 8);
    ctx->last_stats[4] = (long long)st[0];
    ctx->last_stats[5] = (long long)(st[3] | (st[4] << 32));
    ctx->last_stats[6] = (long long)st[2];
    ctx->last_stats[7] = nsrc;
    ctx->last_stats[8] = (long long)st[5];
    ctx->last_stats[9] = (long long)st[6];
    ctx->last_stats[10] = 0;
    ctx->last_stats[11] = (long long)st[7];
    ctx->last_stats[12] = blocks | ((long long)kt << 32) | ((long long)ntpb << 40) | ((long long)fg << 56);
    ctx->last_stats[13] = (long long)st[13];
    ctx->last_stats[14] = (long long)st[14] * g->tvw * 8;   // bytes of tile-visibility rows read
    ctx->last_stats[15] = (long long)st[15];                          // runs scanned in phase C
    ctx->last_stats[16] = (long long)st[1];                           // phase-C cells that hit
    ctx->last_stats[17] = (long long)st[14];                          // phase-C cells (regular)
    ctx->last_stats[35] = (long long)st[30];                          // phase-C partial-tile masks read
    ctx->last_stats[36] = (long long)st[31];                          // phase-C cells tested by masks
    ctx->last_stats[37] = (long long)(g->pmask.p ? g->pmask.n * 8 : 0);  // bytes of partial-tile masks held
    prep_state_stats(ctx, g);
    if (pg) {   // asymmetric mode (bit 7) and |A|
        ctx->last_stats[40] |= 128;
        ctx->last_stats[43] = pg->nasym;
    }
    if (nseeds > 0) return DMX_OK;
    if (!out_on_device && nsrc > 0)
        HIPCHK(copy_sync(ctx->stream, out + sb * 7, d_out.p + sb * 7, nsrc * 7 * 4, hipMemcpyDeviceToHost));
    if (levels && nsrc > 0)
        HIPCHK(copy_sync(ctx->stream, levels + sb * 3, d_lv.p + sb * 3, nsrc * 3 * 8, hipMemcpyDeviceToHost));
    return DMX_OK;
}

// Asymmetric mode (vga_tile.hip): a graph whose runs are not symmetric at scale -- a map re-read from a .graph file,
// where PixelVec's 4-bit row shift (ngraph.cpp:536-583) moved the runs after a jump of more than 15 rows and a bin
// of 65536 k cells lost its runs (Bin::write's unsigned short count) -- has almost every node asymmetric, beyond
// the in-set correction lists.  Made again from the drawing, the map's graph R is symmetric but for a few nodes;
// A = the nodes whose runs differ between the graph and R, plus R's asymmetric nodes.  Every edge between two
// nodes outside A is in both graphs and in both directions, so the search runs bottom-up on R with the frontier
// limited to cells outside A, and the A cells of each frontier push the graph's own runs top-down.  Needs the
// drawing (dmx_graph_set_drawing), the whole graph, no merge links, R on the same grid and |A| <= N/4.
static int prepare_asym(dmx_ctx* ctx, dmx_graph* g) {
    if (g->asym_state) return g->asym_state > 0 ? DMX_OK : DMX_ERR_UNSUPPORTED;
    g->asym_state = -1;
    if (!g->has_drawing) { g->asym_why = "no drawing"; return DMX_ERR_UNSUPPORTED; }
    if (!g->merges.empty()) { g->asym_why = "merge links"; return DMX_ERR_UNSUPPORTED; }
    if (g->node_begin != 0 || g->node_end != g->nnodes) { g->asym_why = "a shard"; return DMX_ERR_UNSUPPORTED; }
    const PointMapHost& h = *g->pm->host;
    std::unique_ptr<dmx_pointmap> pm(new dmx_pointmap());
    pm->host.reset(new PointMapHost(h.parent_region(), h.spacing(), g->drawing.data(), (int64_t)g->drawing.size() / 4));
    PointMapHost& hr = *pm->host;
    if (hr.cols() != h.cols() || hr.rows() != h.rows() || hr.bottom_left().x != h.bottom_left().x ||
        hr.bottom_left().y != h.bottom_left().y) {
        g->asym_why = "the drawing's grid differs from the map's";
        return DMX_ERR_UNSUPPORTED;
    }
    hr.block_lines();
    hr.restore_fill(h.state().data());
    pm->version++;
    const double t0 = now_s();
    // (makeGraph's timing and counters are the reference graph's from here on)
    dmx_graph* r = nullptr;
    if (int rc = makegraph_impl(ctx, pm.get(), -1.0, 0, 0, -1, nullptr, nullptr, &r)) {
        g->asym_why = "makeGraph of the reference failed";
        return rc;
    }
    std::unique_ptr<dmx_graph> R(r);
    if (R->nnodes != g->nnodes) { g->asym_why = "the reference has other nodes"; return DMX_ERR_UNSUPPORTED; }
    if (int rc = prepare_uf(R.get())) return rc;
    if (int rc = prepare_symmetry(R.get())) return rc;
    if (R->symmetric != 1) { g->asym_why = "the reference is not symmetric enough"; return DMX_ERR_UNSUPPORTED; }
    const int64_t N = g->nnodes;
    DevBuf<uint8_t> d_flag;
    HIPCHK(d_flag.alloc(std::max<int64_t>(N, 1)));
    if (N) {
        hipLaunchKernelGGL(node_runs_differ_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, ctx->stream, N,
                           g->bin_nruns.p, g->node_run_start.p, g->node_nruns.p, g->pool.p, R->bin_nruns.p,
                           R->node_run_start.p, R->node_nruns.p, R->pool.p, d_flag.p);
        HIPCHK(hipGetLastError());
    }
    std::vector<uint8_t> flag((size_t)std::max<int64_t>(N, 1));
    HIPCHK(copy_sync(ctx->stream, flag.data(), d_flag.p, (size_t)N, hipMemcpyDeviceToHost));
    for (int32_t k : R->special_nodes) flag[k] = 1;
    const int tw = (h.cols() + 7) / 8, th = (h.rows() + 7) / 8;
    std::vector<unsigned long long> at((size_t)tw * th, 0ull);
    int64_t na = 0;
    for (int64_t k = 0; k < N; k++)
        if (flag[k]) {
            const int c = g->pm->node_cell[k], x = c / h.rows(), y = c % h.rows();
            at[(size_t)(y >> 3) * tw + (x >> 3)] |= 1ull << ((y & 7) * 8 + (x & 7));
            na++;
        }
    if (na > N / 4) { g->asym_why = "too many nodes differ from the reference"; return DMX_ERR_UNSUPPORTED; }
    HIPCHK(g->asym_tiles.alloc(at.size()));
    HIPCHK(copy_sync(ctx->stream, g->asym_tiles.p, at.data(), at.size() * 8, hipMemcpyHostToDevice));
    g->nasym = na;
    g->aref = std::move(R);
    g->aref_pm = std::move(pm);
    g->asym_state = 1;
    VLOG("asymmetric mode: reference graph %.2f s, %lld of %lld nodes differ (%zu asymmetric in the reference)\n",
         now_s() - t0, (long long)na, (long long)N, g->aref->special_nodes.size());
    return DMX_OK;
}

int dmx_graph_set_drawing(dmx_graph* g, const double* lines, int64_t nlines) {
    if (!g || nlines < 0 || (nlines > 0 && !lines)) return fail(DMX_ERR_ARG, "bad arguments");
    g->drawing.assign(lines, lines + 4 * nlines);
    g->has_drawing = true;
    g->asym_state = 0;
    g->aref.reset();
    g->aref_pm.reset();
    g->asym_tiles.reset();
    return DMX_OK;
}

static int vga_impl(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t sb, int64_t se, float* out,
                    bool out_on_device, int64_t* levels) {
    if (!ctx || !g || !out) return fail(DMX_ERR_ARG, "bad arguments");
    if (g->node_begin != 0 || g->node_end != g->nnodes)
        return fail(DMX_ERR_STATE, "VGA needs the whole graph (assemble the shards first)");
    HIPCHK(hipSetDevice(ctx->device));
    const int64_t N = g->nnodes;
    if (se < 0 || se > N) se = N;
    if (sb < 0 || sb > se) return fail(DMX_ERR_ARG, "bad source range");
    int rc = prepare_uf(g);
    if (rc) return rc;
    rc = prepare_symmetry(g);
    if (rc) return rc;
    ctx->last_stats[40] = 0;   // (the tile search sets its preparation flags; the other searches leave none)
    ctx->last_stats[43] = 0;
    PointMapHost& h = *g->pm->host;
    const int tw = (h.cols() + 7) / 8, th = (h.rows() + 7) / 8;
    const int maxlev = 4096;
    {
        const char* fk = getenv("DMX_VGA_KERNEL");
        const bool forced_other = fk && (std::string(fk) == "v1" || std::string(fk) == "do" || std::string(fk) == "topdown");
        const int nt = tw * th;
        // DMX_VGA_ASYM (test hook): the asymmetric mode also for a graph whose few asymmetric nodes the in-set
        // correction lists handle (small re-read maps), so that both exact paths can be compared
        const bool force_asym = getenv("DMX_VGA_ASYM") && g->has_drawing && g->symmetric == 1 && g->nspecial > 0;
        if (!forced_other && g->symmetric == 1 && !ctx->tile_disabled && !force_asym) {
            int rc2 = vga_tile_impl(ctx, g, radius, gates_only, sb, se, out, out_on_device, levels, tw, th);
            if (rc2 != DMX_ERR_CAPACITY) return rc2;   // capacity (level histogram): retry with vga_do
        } else if (!forced_other && (g->symmetric == 0 || force_asym) && !ctx->tile_disabled && !getenv("DMX_VGA_NOASYM") &&
                   prepare_asym(ctx, g) == DMX_OK) {
            // asymmetric at scale (a re-read .graph): the tile search on the reference graph, A pushing its own runs
            int rc2 = vga_tile_impl(ctx, g->aref.get(), radius, gates_only, sb, se, out, out_on_device, levels, tw, th,
                                    nullptr, 0, nullptr, nullptr, g);
            if (rc2 != DMX_ERR_CAPACITY) return rc2;
        }
    }
    if (int rc3 = restore_scan_order(g)) return rc3;   // (vga_do reads the scan order)
    const size_t lds_do = (size_t)tw * th * 8 * 3 + (maxlev + 4) * 4 + 64;
    const char* force = getenv("DMX_VGA_KERNEL");
    const bool want_v1 = force && std::string(force) == "v1";
    const bool gbm = !want_v1 && lds_do > 160 * 1024;   // bitmaps in HBM
    const bool use_do = !want_v1;
    const size_t lds = gbm ? (size_t)(maxlev + 4) * 4 + 64 : use_do ? lds_do : (size_t)tw * th * 8 + (maxlev + 4) * 4 + 64;
    if (lds > 160 * 1024) return fail(DMX_ERR_UNSUPPORTED, "grid too large for the LDS visited bitmap (v1 limit)");
    int occ = 0;
    if (gbm) HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, vga_do_kernel<true>, DO_THREADS, lds));
    else if (use_do) HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, vga_do_kernel<false>, DO_THREADS, lds));
    else HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, vga_global_kernel, VGA_THREADS, lds));
    if (occ < 1) occ = 1;
    const int64_t nsrc = se - sb;
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((int64_t)ctx->num_cu * occ, nsrc));
    DevBuf<int32_t> frontier;
    HIPCHK(frontier.alloc((size_t)blocks * 2 * std::max<int64_t>(N, 1)));
    DevBuf<unsigned long long> gbm_buf;
    if (gbm) HIPCHK(gbm_buf.alloc((size_t)blocks * 3 * tw * th));
    DevBuf<float> d_out;
    float* outp = out;
    if (!out_on_device) {
        HIPCHK(d_out.alloc(std::max<int64_t>(N, 1) * 7));
        outp = d_out.p;
    }
    DevBuf<int64_t> d_lv;
    if (levels) HIPCHK(d_lv.alloc(std::max<int64_t>(N, 1) * 3));
    HIPCHK(hipMemsetAsync(ctx->counters.p, 0, 16 * sizeof(int), ctx->stream));
    HIPCHK(hipMemsetAsync(ctx->stats.p, 0, 32 * sizeof(unsigned long long), ctx->stream));
    VgaParams P;
    P.cols = h.cols(); P.rows = h.rows(); P.tw = tw; P.th = th;
    P.seed_tiles = g->pm->d_seed_tiles.p; P.uf_tiles = g->uf_tiles.p; P.uf_count = g->uf_count;
    P.node_cell = g->pm->d_node_cell.p; P.cell_node = g->pm->d_cell_node.p; P.node_flags = g->pm->d_node_flags.p;
    P.node_run_start = g->node_run_start.p; P.node_nruns = g->node_nruns.p; P.pool = g->pool.p;
    P.src_begin = sb; P.src_end = se; P.radius = (int)radius; P.gates_only = gates_only;
    P.work_counter = ctx->counters.p + 0; P.error = ctx->counters.p + 1;
    P.frontier = frontier.p; P.nnodes = N; P.maxlev = maxlev;
    P.out = outp; P.levels_out = levels ? d_lv.p : nullptr;
    P.stats = ctx->stats.p;
    VgaDoParams Q;
    Q.cols = h.cols(); Q.rows = h.rows(); Q.tw = tw; Q.th = th;
    Q.seed_tiles = g->notuf_tiles.p; Q.uf_tiles = g->uf_tiles.p; Q.nonexp_tiles = g->pm->d_nonexp_tiles.p;
    Q.node_cell = P.node_cell; Q.cell_node = P.cell_node; Q.node_flags = P.node_flags;
    Q.node_run_start = P.node_run_start; Q.node_nruns = P.node_nruns; Q.pool = P.pool;
    Q.cell_scan_start = g->cell_scan_start.p; Q.cell_nruns = g->cell_nruns.p; Q.scan_pool = g->scan_pool.p;
    Q.src_begin = sb; Q.src_end = se; Q.radius = P.radius; Q.gates_only = gates_only;
    Q.uf_count = g->uf_count; Q.symmetric = g->symmetric;
    const bool corr = g->symmetric == 1 && g->nspecial > 0;
    Q.spec_index = corr ? g->spec_index.p : nullptr;
    Q.extra_off = corr ? g->extra_off.p : nullptr;
    Q.extra = corr ? g->extra.p : nullptr;
    Q.missing_off = corr ? g->missing_off.p : nullptr;
    Q.missing = corr ? g->missing.p : nullptr;
    Q.alpha = 15; Q.kshort = 16;
    if (const char* a = getenv("DMX_VGA_ALPHA")) Q.alpha = atoi(a);
    if (const char* k = getenv("DMX_VGA_KSHORT")) Q.kshort = atoi(k);
    Q.work_counter = P.work_counter; Q.scratch = frontier.p; Q.nnodes = N; Q.maxlev = maxlev;
    Q.out = outp; Q.levels_out = P.levels_out; Q.error = P.error; Q.stats = P.stats;
    Q.gbm = gbm ? gbm_buf.p : nullptr;
    Q.nmp = (int)(g->merges.size() / 2);
    Q.mpairs = Q.nmp ? g->d_mpairs.p : nullptr;
    if (!use_do && Q.nmp) return fail(DMX_ERR_UNSUPPORTED, "the top-down v1 kernel does not follow merge links");
    Q.nmamb = Q.nmp && radius != -1.0 ? g->nmamb : 0;
    Q.mamb = Q.nmamb ? g->d_mamb.p : nullptr;
    DevBuf<int32_t> mseen;
    DevBuf<uint8_t> oflag;
    if (Q.nmamb) {
        HIPCHK(mseen.alloc((size_t)blocks * Q.nmamb));
        HIPCHK(hipMemsetAsync(mseen.p, 0, (size_t)blocks * Q.nmamb * 4, ctx->stream));
        Q.mseen = mseen.p;
        HIPCHK(oflag.alloc(N));
        HIPCHK(hipMemsetAsync(oflag.p, 0, (size_t)N, ctx->stream));
        Q.oflag = oflag.p;
    }
    HIPCHK(hipEventRecord(ctx->ev0, ctx->stream));
    if (nsrc > 0) {
        if (gbm) hipLaunchKernelGGL(vga_do_kernel<true>, dim3((unsigned)blocks), dim3(DO_THREADS), lds, ctx->stream, Q);
        else if (use_do) hipLaunchKernelGGL(vga_do_kernel<false>, dim3((unsigned)blocks), dim3(DO_THREADS), lds, ctx->stream, Q);
        else hipLaunchKernelGGL(vga_global_kernel, dim3((unsigned)blocks), dim3(VGA_THREADS), lds, ctx->stream, P);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(ctx->ev1, ctx->stream));
    ctx->h_ctl->progress = 0;   // these kernels do not poll: a cancel takes effect when they finish
    HIPCHK(wait_progress(ctx, DMX_PHASE_VGA, nsrc, 1));
    CANCEL_POINT(ctx);
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->last_vga_s = ms * 1e-3;
    int hc[2];
    HIPCHK(copy_sync(ctx->stream, hc, ctx->counters.p, sizeof(hc), hipMemcpyDeviceToHost));
    if (hc[1] & ~KERR_ORDER) return fail(DMX_ERR_CAPACITY, "VGA BFS exceeded its level/frontier capacity");
    ctx->last_stats[38] = 0;
    if (hc[1] & KERR_ORDER)
        if (int rc2 = vga_order_rerun(ctx, g, radius, oflag.p, outp, P.levels_out)) return rc2;
    unsigned long long st[8];
    HIPCHK(copy_sync(ctx->stream, st, ctx->stats.p, sizeof(st), hipMemcpyDeviceToHost));
    ctx->last_stats[8] = (long long)st[5];   // bottom-up cells that scanned all their runs without a hit
    ctx->last_stats[9] = (long long)st[6];   // runs read by those
    ctx->last_stats[10] = gbm ? 1 : 0;
    for (int i = 13; i < 24; i++) ctx->last_stats[i] = 0;
    ctx->last_stats[3] = (long long)(use_do ? (g->symmetric ? 2 : 1) : 0) | ((long long)g->nspecial << 8);
    ctx->last_stats[4] = (long long)st[0];
    ctx->last_stats[5] = (long long)(st[3] | (st[4] << 32));                 // bottom-up | top-down levels
    ctx->last_stats[6] = (long long)st[2];
    ctx->last_stats[7] = nsrc;
    if (!out_on_device && nsrc > 0)
        HIPCHK(copy_sync(ctx->stream, out + sb * 7, d_out.p + sb * 7, nsrc * 7 * 4, hipMemcpyDeviceToHost));
    if (levels && nsrc > 0)
        HIPCHK(copy_sync(ctx->stream, levels + sb * 3, d_lv.p + sb * 3, nsrc * 3 * 8, hipMemcpyDeviceToHost));
    return DMX_OK;
}

int dmx_vga_global(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t sb, int64_t se, float* out,
                   int64_t* levels) {
    SAME_DEVICE(ctx, g);
    if (int rc = prepare_merges(g)) return rc;
    return vga_impl(ctx, g, radius, gates_only, sb, se, out, false, levels);
}

int dmx_vga_global_device(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t sb, int64_t se,
                          float* out_device) {
    SAME_DEVICE(ctx, g);
    if (int rc = prepare_merges(g)) return rc;
    return vga_impl(ctx, g, radius, gates_only, sb, se, out_device, true, nullptr);
}

// VGA global for an arbitrary set of source nodes (multi-GPU shards interleaved over the grid so that
// every rank gets the same mix of cheap and expensive sources).  The tile-resolved BFS takes the list
// in one launch; otherwise runs of consecutive nodes go through vga_impl one by one.
int dmx_vga_global_device_list(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, const int64_t* nodes,
                               int64_t n, float* out_device) {
    SAME_DEVICE(ctx, g);
    if (!ctx || !g || !out_device || (n > 0 && !nodes)) return fail(DMX_ERR_ARG, "bad arguments");
    if (int rc = prepare_merges(g)) return rc;
    if (g->node_begin != 0 || g->node_end != g->nnodes)
        return fail(DMX_ERR_STATE, "VGA needs the whole graph (assemble the shards first)");
    HIPCHK(hipSetDevice(ctx->device));
    const int64_t N = g->nnodes;
    std::vector<int32_t> lst((size_t)std::max<int64_t>(n, 1));
    for (int64_t i = 0; i < n; i++) {
        if (nodes[i] < 0 || nodes[i] >= N) return fail(DMX_ERR_ARG, "source node out of range");
        lst[i] = (int32_t)nodes[i];
    }
    int rc = prepare_uf(g);
    if (rc) return rc;
    rc = prepare_symmetry(g);
    if (rc) return rc;
    PointMapHost& h = *g->pm->host;
    const int tw = (h.cols() + 7) / 8, th = (h.rows() + 7) / 8;
    if (g->symmetric == 1 && !ctx->tile_disabled) {
        DevBuf<int32_t> d_list;
        HIPCHK(d_list.alloc(lst.size()));
        HIPCHK(hipMemcpyAsync(d_list.p, lst.data(), lst.size() * 4, hipMemcpyHostToDevice, ctx->stream));
        rc = vga_tile_impl(ctx, g, radius, gates_only, 0, n, out_device, true, nullptr, tw, th, nullptr, 0, nullptr, d_list.p);
        if (rc != DMX_ERR_CAPACITY) return rc;
    }
    // Grids above 1024^2, asymmetric graphs or a capacity retry: the other BFS kernels take contiguous
    // source ranges, so each maximal run of consecutive listed nodes is one call (the preparation, and
    // with it every collective of a sharded preparation, is already done: the ranks may differ in the
    // number of calls from here on).  Kernel times add up; the work counters are the last call's.
    const bool was_disabled = ctx->tile_disabled;
    ctx->tile_disabled = true;
    double total = 0.0;
    for (int64_t i = 0; i < n;) {
        int64_t j = i + 1;
        while (j < n && lst[j] == lst[j - 1] + 1) j++;
        rc = vga_impl(ctx, g, radius, gates_only, lst[i], (int64_t)lst[j - 1] + 1, out_device, true, nullptr);
        if (rc) break;
        total += ctx->last_vga_s;
        i = j;
    }
    ctx->tile_disabled = was_disabled;
    if (rc) return rc;
    ctx->last_vga_s = total;
    return DMX_OK;
}

// ---------------------------------------------------------------- VGA metric (all sources)
// VGAMetric::run / VGAAngular::run for every source: one search per workgroup (stepdepth.hip).
extern "C++" template <bool ANG>
static int vga_search_all(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t sb, int64_t se, float* out) {
    constexpr int NO = ANG ? 3 : 4;
    if (!ctx || !g || !out) return fail(DMX_ERR_ARG, "bad arguments");
    if (g->node_begin != 0 || g->node_end != g->nnodes)
        return fail(DMX_ERR_STATE, "VGA needs the whole graph (assemble the shards first)");
    HIPCHK(hipSetDevice(ctx->device));
    PointMapHost& h = *g->pm->host;
    const int cols = h.cols(), rows = h.rows();
    const int64_t C = (int64_t)cols * rows, N = g->nnodes;
    if (se < 0 || se > N) se = N;
    if (sb < 0 || sb > se) return fail(DMX_ERR_ARG, "source range out of bounds");
    const auto& st = h.state();
    // expanders: BLOCKED or next to a BLOCKED cell (ngraph.cpp:67-76, pointdata.cpp:1016-1068); the
    // source expands at distance 0 whatever its flags
    std::vector<uint8_t> flags((size_t)C, 0);
    int64_t nexp = 0;
    for (int x = 0; x < cols; x++)
        for (int y = 0; y < rows; y++) {
            const int64_t c = h.index(x, y);
            if (!(st[c] & CELL_FILLED)) continue;
            uint8_t f = SDF_FILLED;
            bool ex = (st[c] & CELL_BLOCKED) != 0;
            for (int dx = -1; dx <= 1 && !ex; dx++)
                for (int dy = -1; dy <= 1 && !ex; dy++)
                    if ((dx || dy) && h.includes(x + dx, y + dy) && (st[h.index(x + dx, y + dy)] & CELL_BLOCKED)) ex = true;
            if (ex) { f |= SDF_EXPAND; nexp++; }
            flags[c] = f;
        }
    for (size_t i = 0; i < g->merges.size(); i++) { flags[g->merges[i]] |= SDF_MERGE; nexp++; }
    hipStream_t s = ctx->stream;
    int occ = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, vga_metric_kernel<ANG>, SD_THREADS, 0));
    const int64_t nb = std::max<int64_t>(1, std::min<int64_t>(se - sb, (int64_t)ctx->num_cu * std::max(occ, 1)));
    DevBuf<uint8_t> d_flags;
    DevBuf<unsigned long long> d_key, d_over, d_comp, d_srt;
    DevBuf<float> d_mdist, d_cum, d_out;
    DevBuf<int32_t> d_last;
    HIPCHK(d_flags.alloc(C));
    HIPCHK(d_key.alloc((size_t)nb * C));
    HIPCHK(d_mdist.alloc((size_t)nb * C));
    HIPCHK(d_cum.alloc((size_t)nb * C));
    HIPCHK(d_last.alloc((size_t)nb * C));
    HIPCHK(d_comp.alloc((size_t)nb * 2 * std::max<int64_t>(N, 1)));
    HIPCHK(d_srt.alloc((size_t)nb * std::max<int64_t>(N, 1)));
    HIPCHK(d_out.alloc((size_t)std::max<int64_t>(N, 1) * NO));
    HIPCHK(hipMemcpyAsync(d_flags.p, flags.data(), C, hipMemcpyHostToDevice, s));
    // Per-workgroup overflow list.  A source whose search outgrows it stops, is listed, and only the
    // listed sources run again with a 4x list on fewer workgroups (bounded by free device memory).
    int64_t cap = 8 * (nexp + 1) + SD_WIN + 1024;
    if (ANG) cap += 32 * N;   // cells reached at angle 0 are queued too (and re-queued on improvement)
    if (const char* e = getenv("DMX_SD_CAP")) cap = std::max<int64_t>(64, atoll(e));   // test hook: retries
    DevBuf<int64_t> d_list[2];
    DevBuf<int> d_nfail;
    HIPCHK(d_list[0].alloc(std::max<int64_t>(se - sb, 1)));
    HIPCHK(d_list[1].alloc(std::max<int64_t>(se - sb, 1)));
    HIPCHK(d_nfail.alloc(1));
    HIPCHK(hipMemsetAsync(ctx->counters.p, 0, 16 * sizeof(int), s));
    HIPCHK(hipMemsetAsync(ctx->stats.p, 0, 32 * sizeof(unsigned long long), s));
    double kernel_s = 0.0;
    int64_t todo = se - sb, rerun = 0;
    const int64_t* list = nullptr;   // first pass: the range; then the failed sources
    int cur = 0;
    for (int attempt = 0; todo > 0; attempt++) {
        const int64_t nbl = std::max<int64_t>(1, std::min<int64_t>(nb, todo));
        size_t free_b = 0, total_b = 0;
        HIPCHK(hipMemGetInfo(&free_b, &total_b));
        free_b += cached_bytes() + d_over.n * sizeof(unsigned long long);
        const int64_t cap_max = (int64_t)(free_b * 0.8 / 8.0 / (double)nbl);
        if (attempt > 0 && cap > cap_max) return fail(DMX_ERR_CAPACITY, "VGA metric/angular: search queue exceeds device memory");
        if (attempt >= 10) return fail(DMX_ERR_CAPACITY, "VGA metric/angular: queue overflow after retries");
        d_over.reset();
        HIPCHK(d_over.alloc((size_t)nbl * std::min(cap, std::max<int64_t>(cap_max, 1))));
        const int64_t cap_used = std::min(cap, std::max<int64_t>(cap_max, 1));
        HIPCHK(hipMemsetAsync(d_nfail.p, 0, sizeof(int), s));
        StepDepthParams P;
        P.cols = cols; P.rows = rows; P.flags = d_flags.p; P.cell_node = g->pm->d_cell_node.p;
        P.node_run_start = g->node_run_start.p; P.node_nruns = g->node_nruns.p; P.pool = g->pool.p;
        P.key = d_key.p; P.mdist = d_mdist.p; P.cum = d_cum.p; P.lastpix = d_last.p;
        P.over = d_over.p; P.over_cap = cap_used; P.error = ctx->counters.p + 1; P.stats = ctx->stats.p;
        P.merge = g->merges.empty() ? nullptr : g->d_merge_cell.p;
        HIPCHK(hipEventRecord(ctx->ev0, s));
        hipLaunchKernelGGL(vga_metric_kernel<ANG>, dim3((unsigned)nbl), dim3(SD_THREADS), 0, s, P, C, g->pm->d_node_cell.p,
                           list ? 0 : sb, list ? todo : se, gates_only, h.spacing(), radius < 0 ? -1.0 : radius, d_comp.p,
                           d_srt.p, std::max<int64_t>(N, 1), d_out.p, list, d_list[cur].p, d_nfail.p);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(ctx->ev1, s));
        HIPCHK(hipStreamSynchronize(s));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
        kernel_s += ms * 1e-3;
        int hc[2], nfail = 0;
        HIPCHK(copy_sync(ctx->stream, hc, ctx->counters.p, sizeof(hc), hipMemcpyDeviceToHost));
        HIPCHK(copy_sync(ctx->stream, &nfail, d_nfail.p, sizeof(int), hipMemcpyDeviceToHost));
        if (hc[1] & ~KERR_FRONTIER) return fail(DMX_ERR_CAPACITY, "VGA metric/angular search failed");
        VLOG("vga %s: attempt %d, %lld sources, list %lld per workgroup x %lld: %.3f s, %d to re-run\n",
             ANG ? "angular" : "metric", attempt, (long long)todo, (long long)cap_used, (long long)nbl, ms * 1e-3, nfail);
        if (nfail > 0 && cap_used < cap) return fail(DMX_ERR_CAPACITY, "VGA metric/angular: search queue exceeds device memory");
        HIPCHK(hipMemsetAsync(ctx->counters.p + 1, 0, sizeof(int), s));
        rerun += nfail;
        todo = nfail;
        list = d_list[cur].p;
        cur ^= 1;
        cap *= 4;
    }
    ctx->last_vga_s = kernel_s;   // every attempt counted
    if (se > sb)
        HIPCHK(copy_sync(ctx->stream, out + sb * NO, d_out.p + sb * NO, (size_t)(se - sb) * NO * 4, hipMemcpyDeviceToHost));
    unsigned long long stv[3];
    HIPCHK(copy_sync(ctx->stream, stv, ctx->stats.p, sizeof(stv), hipMemcpyDeviceToHost));
    ctx->last_sd_stats[0] = (long long)stv[0];
    ctx->last_sd_stats[1] = (long long)stv[1];
    ctx->last_stats[7] = se - sb;
    ctx->last_stats[8] = rerun;   // sources re-run with a larger overflow list
    return DMX_OK;
}

// The symmetry scatter a whole-graph makeGraph did as it published (sym_diff 4*C*8 B, sym_ho N*8 B: ~160 MB at
// 2000^2) serves only the VGA BFS's preparation.  The analyses that do not use it release it; a VGA call after
// them runs the separate scatter pass instead (prepare_symmetry).
static void release_sym_scatter(dmx_graph* g) {
    if (g && g->sym_fused && !g->scan_ready) {
        g->sym_diff.reset();
        g->sym_ho.reset();
        g->sym_fused = false;
    }
}

int dmx_vga_metric(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t sb, int64_t se, float* out) {
    SAME_DEVICE(ctx, g);
    release_sym_scatter(g);
    if (int rc = prepare_merges(g)) return rc;
    return vga_search_all<false>(ctx, g, radius, gates_only, sb, se, out);
}

int dmx_vga_angular(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t sb, int64_t se, float* out) {
    SAME_DEVICE(ctx, g);
    release_sym_scatter(g);
    if (int rc = prepare_merges(g)) return rc;
    return vga_search_all<true>(ctx, g, radius, gates_only, sb, se, out);
}

// ---------------------------------------------------------------- VGA visual local
int dmx_vga_local(dmx_ctx* ctx, dmx_graph* g, int gates_only, int64_t sb, int64_t se, float* out) {
    SAME_DEVICE(ctx, g);
    release_sym_scatter(g);
    if (!ctx || !g || !out) return fail(DMX_ERR_ARG, "bad arguments");
    if (g->node_begin != 0 || g->node_end != g->nnodes)
        return fail(DMX_ERR_STATE, "VGA needs the whole graph (assemble the shards first)");
    HIPCHK(hipSetDevice(ctx->device));
    const int64_t N = g->nnodes;
    if (se < 0 || se > N) se = N;
    if (sb < 0 || sb > se) return fail(DMX_ERR_ARG, "source range out of bounds");
    PointMapHost& h = *g->pm->host;
    const int cols = h.cols(), rows = h.rows();
    const int tw = (cols + 7) / 8, th = (rows + 7) / 8, nt = tw * th;
    const size_t bm_bytes = (size_t)2 * nt * 8;
    const bool gbm = bm_bytes > 150 * 1024 || getenv("DMX_VL_GBM");   // the env forces the HBM variant (tests)
    const size_t lds = gbm ? 0 : bm_bytes;
    hipStream_t s = ctx->stream;
    DevBuf<int32_t> nsz;
    DevBuf<float> d_out;
    DevBuf<unsigned long long> d_bm;
    HIPCHK(nsz.alloc(std::max<int64_t>(N, 1)));
    HIPCHK(d_out.alloc((size_t)std::max<int64_t>(N, 1) * 3));
    HIPCHK(hipMemsetAsync(ctx->stats.p, 0, 32 * 8, s));
    HIPCHK(hipEventRecord(ctx->ev0, s));
    if (se > sb) {
        hipLaunchKernelGGL(node_size_kernel, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, s, N, g->node_run_start.p,
                           g->node_nruns.p, g->pool.p, nsz.p);
        HIPCHK(hipGetLastError());
        int occ = 0;
        auto kern = gbm ? vga_local_kernel<true> : vga_local_kernel<false>;
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, VL_THREADS, lds));
        int64_t nb = std::min<int64_t>(se - sb, (int64_t)ctx->num_cu * std::max(occ, 1));
        if (gbm) {
            // bitmap slices within a quarter of the free memory
            size_t fr = 0, tot = 0;
            HIPCHK(hipMemGetInfo(&fr, &tot));
            nb = std::max<int64_t>(1, std::min<int64_t>(nb, (int64_t)((fr + cached_bytes()) / 4 / bm_bytes)));
            HIPCHK(d_bm.alloc((size_t)nb * 2 * nt));
        }
        hipLaunchKernelGGL(kern, dim3((unsigned)nb), dim3(VL_THREADS), lds, s, cols, rows, tw, th,
                           g->pm->d_node_cell.p, g->pm->d_cell_node.p, g->pm->d_node_flags.p, g->node_run_start.p,
                           g->node_nruns.p, g->pool.p, nsz.p, sb, se, gates_only, d_out.p, ctx->stats.p, d_bm.p);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(ctx->ev1, s));
    HIPCHK(hipStreamSynchronize(s));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->last_vga_s = ms * 1e-3;
    if (se > sb)
        HIPCHK(copy_sync(ctx->stream, out + sb * 3, d_out.p + sb * 3, (size_t)(se - sb) * 3 * 4, hipMemcpyDeviceToHost));
    unsigned long long st0 = 0;
    HIPCHK(copy_sync(ctx->stream, &st0, ctx->stats.p, 8, hipMemcpyDeviceToHost));
    ctx->last_stats[4] = (long long)st0;   // neighbour runs walked
    ctx->last_stats[7] = se - sb;
    return DMX_OK;
}

int dmx_graph_set_prep_shard(dmx_graph* g, int64_t node_begin, int64_t node_end, dmx_allreduce_fn fn, void* user) {
    if (!g) return fail(DMX_ERR_ARG, "bad arguments");
    if (fn && (node_begin < 0 || node_end < node_begin || node_end > g->nnodes))
        return fail(DMX_ERR_ARG, "prep node range out of bounds");
    if (g->uf_count >= 0 || g->symmetric >= 0 || g->tiles_ready)
        return fail(DMX_ERR_STATE, "VGA preparation already done on this graph");
    g->prep_fn = fn;
    g->prep_user = fn ? user : nullptr;
    g->prep_b = fn ? node_begin : 0;
    g->prep_e = fn ? node_end : -1;
    return DMX_OK;
}

// ---------------------------------------------------------------- metric step depth
// Batched metric search (stepdepth.hip): key/mdist/cum/lastpix are left in the VGAMetricDepth end
// state.  Returns DMX_OK, a negative status on a HIP error, or 1 when a batch capacity overflowed
// (the caller then re-runs the selection with the serial kernel).
static int stepdepth_batched(dmx_ctx* ctx, dmx_graph* g, const std::vector<uint8_t>& flags,
                             const std::vector<int32_t>& sel, const uint8_t* d_flags, const int32_t* d_sel,
                             unsigned long long* d_key, float* d_mdist, float* d_cum, int32_t* d_last) {
    PointMapHost& h = *g->pm->host;
    const int rows = h.rows();
    const int64_t C = (int64_t)h.cols() * rows;
    hipStream_t s = ctx->stream;
    std::vector<int32_t> ex;
    for (int64_t c = 0; c < C; c++)
        if (flags[(size_t)c] & SDF_EXPAND) ex.push_back((int32_t)c);
    const int64_t E = (int64_t)ex.size();
    // work units: ceil(runs / SDB_UNIT) per expander
    std::vector<int32_t> nr((size_t)g->nnodes);
    HIPCHK(hipStreamSynchronize(s));
    if (g->nnodes) HIPCHK(copy_sync(ctx->stream, nr.data(), g->node_nruns.p, g->nnodes * 4, hipMemcpyDeviceToHost));
    int64_t units = 0;
    const auto& nc = g->pm->node_cell;   // ascending cell index = node order
    for (int32_t c : ex) {
        const size_t node = (size_t)(std::lower_bound(nc.begin(), nc.end(), c) - nc.begin());
        units += (nr[node] + SDB_UNIT - 1) / SDB_UNIT;
    }
    const unsigned amb_cap = 1u << 16, ent_cap = 1u << 22;
    DevBuf<int32_t> d_ex, d_uown, d_win, d_ambid, d_touch, d_amb, d_ahead, d_enext;
    DevBuf<uint8_t> d_done;
    DevBuf<SdbExp> d_bq;
    DevBuf<unsigned long long> d_best;
    DevBuf<unsigned> d_nnear;
    DevBuf<int2> d_ent;
    DevBuf<SdbCtl> d_ctl;
    HIPCHK(d_ex.alloc(std::max<int64_t>(E, 1)));
    HIPCHK(d_done.alloc(std::max<int64_t>(E, 1)));
    HIPCHK(d_bq.alloc(std::max<int64_t>(E, 1)));
    HIPCHK(d_uown.alloc(std::max<int64_t>(units, 1)));
    HIPCHK(d_best.alloc(C));
    HIPCHK(d_nnear.alloc(C));
    HIPCHK(d_win.alloc(C));
    HIPCHK(d_ambid.alloc(C));
    HIPCHK(d_touch.alloc(C));
    HIPCHK(d_amb.alloc(amb_cap));
    HIPCHK(d_ent.alloc(ent_cap));
    HIPCHK(d_ahead.alloc(amb_cap));
    HIPCHK(d_enext.alloc(ent_cap));
    HIPCHK(hipMemsetAsync(d_ahead.p, 0xFF, (size_t)amb_cap * 4, s));
    HIPCHK(d_ctl.alloc(1));
    if (E) HIPCHK(hipMemcpyAsync(d_ex.p, ex.data(), E * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(d_done.p, 0, std::max<int64_t>(E, 1), s));
    HIPCHK(hipMemsetAsync(d_best.p, 0xFF, C * 8, s));
    HIPCHK(hipMemsetAsync(d_nnear.p, 0, C * 4, s));
    HIPCHK(hipMemsetAsync(d_ambid.p, 0xFF, C * 4, s));
    HIPCHK(hipMemsetAsync(d_key, 0xFF, C * 8, s));
    std::vector<float> m1((size_t)C, -1.0f);
    HIPCHK(hipMemcpyAsync(d_mdist, m1.data(), C * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(d_cum, 0, C * 4, s));
    HIPCHK(hipMemsetAsync(d_last, 0xFF, C * 4, s));
    SdbCtl c0;
    memset(&c0, 0, sizeof(c0));
    c0.gcur = 0ull;            // the selected cells' distance 0
    c0.gnext = SD_INF;
    HIPCHK(hipMemcpyAsync(d_ctl.p, &c0, sizeof(c0), hipMemcpyHostToDevice, s));
    SdbParams P;
    P.rows = rows; P.E = E; P.flags = d_flags; P.cell_node = g->pm->d_cell_node.p;
    P.node_run_start = g->node_run_start.p; P.node_nruns = g->node_nruns.p; P.pool = g->pool.p;
    P.key = d_key; P.mdist = d_mdist; P.cum = d_cum; P.lastpix = d_last;
    P.ex_cells = d_ex.p; P.ex_done = d_done.p; P.bq = d_bq.p; P.uown = d_uown.p;
    P.best = d_best.p; P.nnear = d_nnear.p; P.win = d_win.p; P.ambid = d_ambid.p; P.touch = d_touch.p;
    P.amb = d_amb.p; P.ent = d_ent.p; P.ahead = d_ahead.p; P.enext = d_enext.p; P.ent_cap = ent_cap; P.amb_cap = amb_cap; P.ctl = d_ctl.p;
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipEventRecord(ctx->ev0, s));
    hipLaunchKernelGGL(sdb_init_kernel, dim3((unsigned)((sel.size() + 255) / 256)), dim3(256), 0, s, P, d_sel,
                       (int)sel.size());
    HIPCHK(hipGetLastError());
    const unsigned gs = (unsigned)std::max<int64_t>(1, (E + 255) / 256);
    const unsigned gr = (unsigned)std::max(64, ctx->num_cu * 4);
    SdbCtl hc;
    // Batches advance the smallest live distance by >= 1 - 2^-18; the number of batches is bounded
    // by the longest path length, itself < C grid units.
    const int64_t max_it = 2 * C + 64;
    int64_t it = 0;
    for (;;) {
        for (int k = 0; k < 32; k++, it++) {
            hipLaunchKernelGGL(sdb_select_kernel, dim3(gs), dim3(256), 0, s, P);
            hipLaunchKernelGGL(sdb_relax_kernel<1>, dim3(gr), dim3(SDB_THREADS), 0, s, P);
            hipLaunchKernelGGL(sdb_relax_kernel<2>, dim3(gr), dim3(SDB_THREADS), 0, s, P);
            hipLaunchKernelGGL(sdb_apply_kernel, dim3(gr), dim3(256), 0, s, P);
            hipLaunchKernelGGL(sdb_relax_kernel<3>, dim3(gr), dim3(SDB_THREADS), 0, s, P);
            hipLaunchKernelGGL(sdb_fold_kernel, dim3(256), dim3(SDB_THREADS), 0, s, P);
            hipLaunchKernelGGL(sdb_finish_kernel, dim3(1), dim3(1), 0, s, P);
        }
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(&hc, d_ctl.p, sizeof(hc), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (hc.done) break;
        CANCEL_POINT(ctx);
        if (it > max_it) return fail(DMX_ERR_STATE, "batched step depth did not terminate");
    }
    HIPCHK(hipEventRecord(ctx->ev1, s));
    HIPCHK(hipEventSynchronize(ctx->ev1));
    if (hc.error) return 1;
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->last_sd_s = ms * 1e-3;
    ctx->last_sd_stats[0] = (long long)hc.popped;
    ctx->last_sd_stats[1] = (long long)hc.relaxed;
    ctx->last_sd_stats[2] = (long long)hc.batches;
    ctx->last_sd_extra[0] = (long long)hc.improved;
    ctx->last_sd_extra[1] = (long long)hc.ambiguous;
    return DMX_OK;
}

// STEPDEPTH -sdt metric (VGAMetricDepth) or, with ANG, -sdt angular (VGAAngularDepth): one search
// from the selection; out [N][3] (metric) or [N] (angular).
extern "C++" template <bool ANG>
static int stepdepth_impl(dmx_ctx* ctx, dmx_graph* g, const int32_t* sel_cells, int64_t nsel, float* out) {
    if (!ctx || !g || !out || (nsel > 0 && !sel_cells)) return fail(DMX_ERR_ARG, "bad arguments");
    if (g->node_begin != 0 || g->node_end != g->nnodes)
        return fail(DMX_ERR_STATE, "step depth needs the whole graph (assemble the shards first)");
    HIPCHK(hipSetDevice(ctx->device));
    CANCEL_POINT(ctx);   // a cancel requested while nothing ran stops this call (dmx.h)
    PointMapHost& h = *g->pm->host;
    const int cols = h.cols(), rows = h.rows();
    const int64_t C = (int64_t)cols * rows, N = g->nnodes;
    const auto& st = h.state();
    // selection: filled cells only, std::set<int> PixelRef order, no duplicates
    std::vector<int32_t> sel;
    for (int64_t i = 0; i < nsel; i++) {
        const int32_t c = sel_cells[i];
        if (c < 0 || c >= C) return fail(DMX_ERR_ARG, "selected cell outside the grid");
        if (st[c] & CELL_FILLED) sel.push_back(c);
    }
    std::sort(sel.begin(), sel.end(), [&](int32_t a, int32_t b) {
        return ((a / rows) << 16) + (a % rows) < ((b / rows) << 16) + (b % rows);
    });
    sel.erase(std::unique(sel.begin(), sel.end()), sel.end());
    if (sel.empty()) return fail(DMX_ERR_STATE, "no filled cell selected");
    // expanders: selected, BLOCKED or next to a BLOCKED cell (ngraph.cpp:67-76, pointdata.cpp:1016-1068)
    std::vector<uint8_t> flags((size_t)C, 0);
    int64_t nexp = 0;
    for (int x = 0; x < cols; x++)
        for (int y = 0; y < rows; y++) {
            const int64_t c = h.index(x, y);
            if (!(st[c] & CELL_FILLED)) continue;
            uint8_t f = SDF_FILLED;
            bool ex = (st[c] & CELL_BLOCKED) != 0;
            for (int dx = -1; dx <= 1 && !ex; dx++)
                for (int dy = -1; dy <= 1 && !ex; dy++)
                    if ((dx || dy) && h.includes(x + dx, y + dy) && (st[h.index(x + dx, y + dy)] & CELL_BLOCKED)) ex = true;
            if (ex) { f |= SDF_EXPAND; nexp++; }
            flags[c] = f;
        }
    for (int32_t c : sel) flags[c] |= SDF_EXPAND;
    for (size_t i = 0; i < g->merges.size(); i++) { flags[g->merges[i]] |= SDF_MERGE; nexp++; }
    hipStream_t s = ctx->stream;
    DevBuf<uint8_t> d_flags;
    DevBuf<unsigned long long> d_key, d_over;
    DevBuf<float> d_mdist, d_cum, d_out;
    DevBuf<int32_t> d_last, d_sel;
    HIPCHK(d_flags.alloc(C));
    HIPCHK(d_key.alloc(C));
    HIPCHK(d_mdist.alloc(C));
    HIPCHK(d_cum.alloc(C));
    HIPCHK(d_last.alloc(C));
    HIPCHK(d_sel.alloc(sel.size()));
    HIPCHK(d_out.alloc(std::max<int64_t>(N, 1) * 3));
    HIPCHK(hipMemcpyAsync(d_flags.p, flags.data(), C, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_sel.p, sel.data(), sel.size() * 4, hipMemcpyHostToDevice, s));
    int64_t cap = 8 * (nexp + (int64_t)sel.size()) + SD_WIN + 1024 + (ANG ? 8 * N : 0);
    // metric: the batched search over the whole GPU (stepdepth.hip, "batched metric step depth");
    // DMX_SD_KERNEL=serial forces the one-workgroup kernel, which is also the fallback
    // (merge links: the serial kernel, which extracts a partner at its link's pop)
    bool batched = !ANG && g->merges.empty();
    if (const char* e = getenv("DMX_SD_KERNEL")) batched = batched && strcmp(e, "serial") != 0;
    ctx->last_sd_mode = 0;
    if (batched) {
        int rc = stepdepth_batched(ctx, g, flags, sel, d_flags.p, d_sel.p, d_key.p, d_mdist.p, d_cum.p, d_last.p);
        if (rc < 0) return rc;
        if (rc == DMX_OK) {
            const int single = sel.size() == 1 ? 1 : 0;
            if (N) {
                hipLaunchKernelGGL(stepdepth_out_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, rows,
                                   h.spacing(), g->pm->d_node_cell.p, N, d_key.p, d_cum.p, single, sel[0] / rows,
                                   sel[0] % rows, d_out.p);
                HIPCHK(hipGetLastError());
                HIPCHK(hipMemcpyAsync(out, d_out.p, N * 3 * 4, hipMemcpyDeviceToHost, s));
                HIPCHK(hipStreamSynchronize(s));
            }
            ctx->last_sd_mode = 1;
            return DMX_OK;
        }
        // rc > 0: a batch capacity overflowed; the serial search below redoes the whole selection
        ctx->last_sd_mode = 2;
    }
    for (int attempt = 0; attempt < 4; attempt++) {
        HIPCHK(d_over.alloc(cap));
        HIPCHK(hipMemsetAsync(d_key.p, 0xFF, C * 8, s));
        std::vector<float> m1((size_t)C, -1.0f);
        HIPCHK(hipMemcpyAsync(d_mdist.p, m1.data(), C * 4, hipMemcpyHostToDevice, s));
        if (ANG) HIPCHK(hipMemcpyAsync(d_cum.p, m1.data(), C * 4, hipMemcpyHostToDevice, s));
        else HIPCHK(hipMemsetAsync(d_cum.p, 0, C * 4, s));
        HIPCHK(hipMemsetAsync(d_last.p, 0xFF, C * 4, s));
        HIPCHK(hipMemsetAsync(ctx->counters.p, 0, 16 * sizeof(int), s));
        HIPCHK(hipMemsetAsync(ctx->stats.p, 0, 32 * sizeof(unsigned long long), s));
        StepDepthParams P;
        P.cols = cols; P.rows = rows; P.flags = d_flags.p; P.cell_node = g->pm->d_cell_node.p;
        P.node_run_start = g->node_run_start.p; P.node_nruns = g->node_nruns.p; P.pool = g->pool.p;
        P.key = d_key.p; P.mdist = d_mdist.p; P.cum = d_cum.p; P.lastpix = d_last.p;
        P.over = d_over.p; P.over_cap = cap; P.error = ctx->counters.p + 1; P.stats = ctx->stats.p;
        P.merge = g->merges.empty() ? nullptr : g->d_merge_cell.p;
        HIPCHK(hipEventRecord(ctx->ev0, s));
        hipLaunchKernelGGL(stepdepth_kernel<ANG>, dim3(1), dim3(SD_THREADS), 0, s, P, d_sel.p, (int)sel.size());
        HIPCHK(hipGetLastError());
        const int single = sel.size() == 1 ? 1 : 0;
        if (!ANG) {
            hipLaunchKernelGGL(stepdepth_out_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, rows,
                               h.spacing(), g->pm->d_node_cell.p, N, d_key.p, d_cum.p, single, sel[0] / rows,
                               sel[0] % rows, d_out.p);
            HIPCHK(hipGetLastError());
        }
        HIPCHK(hipEventRecord(ctx->ev1, s));
        HIPCHK(hipStreamSynchronize(s));
        int hc[2];
        HIPCHK(copy_sync(ctx->stream, hc, ctx->counters.p, sizeof(hc), hipMemcpyDeviceToHost));
        if (hc[1] & KERR_FRONTIER) { cap *= 4; continue; }
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
        ctx->last_sd_s = ms * 1e-3;
        unsigned long long st3[3];
        HIPCHK(copy_sync(ctx->stream, st3, ctx->stats.p, sizeof(st3), hipMemcpyDeviceToHost));
        for (int i = 0; i < 3; i++) ctx->last_sd_stats[i] = (long long)st3[i];
        if (ANG) {
            // "Angular Step Depth" = m_cumangle of every cell the search resolved (vgaangulardepth.cpp:53-55)
            std::vector<unsigned long long> kh((size_t)C);
            std::vector<float> ch((size_t)C);
            HIPCHK(copy_sync(ctx->stream, kh.data(), d_key.p, C * 8, hipMemcpyDeviceToHost));
            HIPCHK(copy_sync(ctx->stream, ch.data(), d_cum.p, C * 4, hipMemcpyDeviceToHost));
            for (int64_t k = 0; k < N; k++) {
                const int c = g->pm->node_cell[k];
                out[k] = kh[c] != SD_INF ? ch[c] : -1.0f;
            }
        } else if (N) {
            HIPCHK(copy_sync(ctx->stream, out, d_out.p, N * 3 * 4, hipMemcpyDeviceToHost));
        }
        return DMX_OK;
    }
    return fail(DMX_ERR_CAPACITY, "step depth queue overflow after retries");
}

int dmx_metric_stepdepth(dmx_ctx* ctx, dmx_graph* g, const int32_t* sel_cells, int64_t nsel, float* out) {
    SAME_DEVICE(ctx, g);
    release_sym_scatter(g);
    if (int rc = prepare_merges(g)) return rc;
    return stepdepth_impl<false>(ctx, g, sel_cells, nsel, out);
}

int dmx_angular_stepdepth(dmx_ctx* ctx, dmx_graph* g, const int32_t* sel_cells, int64_t nsel, float* out) {
    SAME_DEVICE(ctx, g);
    release_sym_scatter(g);
    if (int rc = prepare_merges(g)) return rc;
    return stepdepth_impl<true>(ctx, g, sel_cells, nsel, out);
}

// The nodes the symmetry pass found asymmetric (their in-set differs from their run-length out-set; the
// BFS kernels route them through exact Extra / Missing lists).  Runs the VGA preparation if needed.
int dmx_graph_special_nodes(dmx_graph* g, int32_t* nodes, int64_t* n) {
    if (!g || !n) return fail(DMX_ERR_ARG, "bad arguments");
    if (g->node_begin != 0 || g->node_end != g->nnodes) return fail(DMX_ERR_STATE, "needs the whole graph");
    HIPCHK(hipSetDevice(g->ctx->device));
    if (int rc = prepare_uf(g)) return rc;
    if (int rc = prepare_symmetry(g)) return rc;
    const int64_t m = (int64_t)g->special_nodes.size();
    if (nodes) {
        if (*n < m) return fail(DMX_ERR_ARG, "buffer too small");
        std::memcpy(nodes, g->special_nodes.data(), (size_t)m * 4);
    }
    *n = m;
    return DMX_OK;
}

int dmx_ctx_last_mk_reruns(dmx_ctx* ctx, int64_t* nodes, int64_t cap, int64_t* n) {
    if (!ctx || !n || cap < 0 || (cap > 0 && !nodes)) return fail(DMX_ERR_ARG, "bad arguments");
    *n = (int64_t)ctx->last_mk_reruns.size();
    for (int64_t i = 0; i < *n && i < cap; i++) nodes[i] = ctx->last_mk_reruns[(size_t)i];
    return DMX_OK;
}

int dmx_ctx_last_phase_cycles(dmx_ctx* ctx, int64_t* out5) {
    if (!ctx || !out5) return fail(DMX_ERR_ARG, "bad arguments");
    for (int i = 0; i < 5; i++) out5[i] = ctx->phase_cycles[i];
    return DMX_OK;
}

// STEPDEPTH -sdt visual: MetaGraph::analyseGraph(point_depth_selection = 1) -> VGAVisualGlobalDepth::run
// (depthmapXcli/runmethods.cpp:767-769, salalib/vgamodules/vgavisualglobaldepth.cpp:23-77).  One
// breadth-first search from every selected filled cell at once (level 0, always expanded); cells are
// discovered through run membership (Bin::extractUnseen, ngraph.cpp:308-326: set semantics, the
// extent short-cut only skips already-covered suffixes); contextfilled odd cells get their level but
// are not expanded.  Runs on the tile-resolved BFS in seed mode (one workgroup).
// Visual step depth for grids above 1024^2 or asymmetric graphs: the level-synchronous top-down
// search of kernels/vstep.hip over the whole GPU.
static int visual_stepdepth_topdown(dmx_ctx* ctx, dmx_graph* g, const std::vector<int32_t>& seeds, int tw, int th,
                                    float* out, const std::vector<int32_t>& sel_cells) {
    PointMapHost& h = *g->pm->host;
    const int rows = h.rows();
    const int64_t C = h.cells(), N = g->nnodes, nt = (int64_t)tw * th;
    hipStream_t s = ctx->stream;
    DevBuf<unsigned long long> vis, cnt;
    DevBuf<int32_t> level, fr[2], pend[2];
    DevBuf<int> err;
    HIPCHK(vis.alloc(nt));
    HIPCHK(cnt.alloc(2));   // next frontier, pending extractions
    HIPCHK(err.alloc(1));
    HIPCHK(hipMemsetAsync(err.p, 0, sizeof(int), ctx->stream));
    const int nmp = (int)(g->merges.size() / 2);
    if (g->nmamb) {
        HIPCHK(pend[0].alloc(g->nmamb));
        HIPCHK(pend[1].alloc(g->nmamb));
    }
    HIPCHK(level.alloc(C));
    HIPCHK(fr[0].alloc(std::max<int64_t>(N, 1)));
    HIPCHK(fr[1].alloc(std::max<int64_t>(N, 1)));
    std::vector<unsigned long long> v0((size_t)nt, 0ull);
    std::vector<int32_t> lv((size_t)C, -1);
    for (int32_t k : seeds) {
        const int c = g->pm->node_cell[k], x = c / rows, y = c % rows;
        v0[(size_t)(y >> 3) * tw + (x >> 3)] |= 1ull << ((y & 7) * 8 + (x & 7));
        lv[c] = 0;
    }
    HIPCHK(hipMemcpyAsync(vis.p, v0.data(), nt * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(level.p, lv.data(), C * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(fr[0].p, seeds.data(), seeds.size() * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipEventRecord(ctx->ev0, s));
    int64_t nf = (int64_t)seeds.size(), npend = 0;
    int cur = 0, L = 0;
    while (nf > 0) {
        HIPCHK(hipMemsetAsync(cnt.p, 0, 16, s));
        const int64_t blocks = std::min<int64_t>((nf + 3) / 4, (int64_t)ctx->num_cu * 16);
        hipLaunchKernelGGL(vsd_level_kernel, dim3((unsigned)blocks), dim3(VSD_THREADS), 0, s, rows, tw,
                           (const int32_t*)fr[cur].p, nf, g->node_run_start.p, g->node_nruns.p, g->pool.p,
                           g->pm->d_cell_node.p, g->pm->d_node_flags.p, L + 1, vis.p, level.p, fr[cur ^ 1].p, cnt.p);
        HIPCHK(hipGetLastError());
        if (nmp) {
            hipLaunchKernelGGL(vsd_merge_kernel, dim3((unsigned)((nmp + 255) / 256)), dim3(256), 0, s, rows, tw,
                               (const int2*)g->d_mpairs.p, nmp, g->pm->d_cell_node.p, g->pm->d_node_flags.p, L + 1,
                               vis.p, level.p, fr[cur ^ 1].p, cnt.p, pend[cur ^ 1].p, cnt.p + 1);
            HIPCHK(hipGetLastError());
        }
        if (npend) {   // the previous level's pending extractions, now that this level is complete
            hipLaunchKernelGGL(vsd_pending_kernel, dim3((unsigned)((npend + 3) / 4)), dim3(VSD_THREADS), 0, s, rows, tw,
                               (const int32_t*)pend[cur].p, npend, g->node_run_start.p, g->node_nruns.p, g->pool.p,
                               g->pm->d_cell_node.p, (const unsigned long long*)vis.p, err.p);
            HIPCHK(hipGetLastError());
        }
        unsigned long long n_next[2] = {0, 0};
        HIPCHK(copy_sync(s, n_next, cnt.p, 16, hipMemcpyDeviceToHost));
        cur ^= 1;
        nf = (int64_t)n_next[0];
        npend = (int64_t)n_next[1];
        L++;
    }
    int herr = 0;
    HIPCHK(copy_sync(s, &herr, err.p, sizeof(int), hipMemcpyDeviceToHost));
    HIPCHK(hipEventRecord(ctx->ev1, s));
    if (herr & KERR_ORDER) {
        // an unexpanded link end whose extraction depends on the pop order reached an unseen cell: the whole
        // search in the reference's order (vga_ordered.hip), from the selection in PixelRef order
        HIPCHK(hipMemsetAsync(level.p, 0xFF, C * 4, s));
        if (int rc = ordered_search(ctx, g, -1.0, {}, sel_cells, nullptr, nullptr, level.p)) return rc;
        HIPCHK(hipEventRecord(ctx->ev1, s));
        ctx->last_stats[38] = 1;
    } else {
        ctx->last_stats[38] = 0;
    }
    HIPCHK(copy_sync(s, lv.data(), level.p, C * 4, hipMemcpyDeviceToHost));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->last_vga_s = ms * 1e-3;
    for (int64_t k = 0; k < N; k++) {
        const int v = lv[g->pm->node_cell[k]];
        out[k] = v >= 0 ? (float)v : -1.0f;
    }
    VLOG("visual step depth: top-down, %d levels, %.3f s\n", L, ms * 1e-3);
    return DMX_OK;
}

int dmx_visual_stepdepth(dmx_ctx* ctx, dmx_graph* g, const int32_t* sel_cells, int64_t nsel, float* out) {
    SAME_DEVICE(ctx, g);
    if (!ctx || !g || !out || (nsel > 0 && !sel_cells)) return fail(DMX_ERR_ARG, "bad arguments");
    if (int rc = prepare_merges(g)) return rc;
    if (g->node_begin != 0 || g->node_end != g->nnodes)
        return fail(DMX_ERR_STATE, "step depth needs the whole graph (assemble the shards first)");
    HIPCHK(hipSetDevice(ctx->device));
    CANCEL_POINT(ctx);   // (before any output is written)
    PointMapHost& h = *g->pm->host;
    const int cols = h.cols(), rows = h.rows();
    const int64_t C = (int64_t)cols * rows, N = g->nnodes;
    for (int64_t k = 0; k < N; k++) out[k] = -1.0f;
    ctx->last_stats[38] = 0;
    const auto& st = h.state();
    std::vector<int32_t> seeds;   // nodes, selection order = std::set<int> PixelRef order, unique
    std::vector<int32_t> sel;     // the selected filled cells in that order
    {
        for (int64_t i = 0; i < nsel; i++) {
            const int32_t c = sel_cells[i];
            if (c < 0 || c >= C) return fail(DMX_ERR_ARG, "selected cell outside the grid");
            if (st[c] & CELL_FILLED) sel.push_back(c);
        }
        std::sort(sel.begin(), sel.end());
        sel.erase(std::unique(sel.begin(), sel.end()), sel.end());
        const auto& nc = g->pm->node_cell;   // ascending x-major cell index = node order
        for (int32_t c : sel) {
            const auto it = std::lower_bound(nc.begin(), nc.end(), c);
            if (it != nc.end() && *it == c) seeds.push_back((int32_t)(it - nc.begin()));
        }
    }
    if (seeds.empty()) return fail(DMX_ERR_STATE, "no filled cell selected");
    // a selected cell's merge pixel takes level 0 and is extracted with it (vgavisualglobaldepth.cpp:55-63)
    if (!g->merges.empty()) {
        const auto& nc = g->pm->node_cell;
        std::vector<int32_t> add;
        for (size_t i = 0; i < g->merges.size(); i += 2) {
            const int32_t a = g->merges[i], b = g->merges[i + 1];
            const int32_t na = (int32_t)(std::lower_bound(nc.begin(), nc.end(), a) - nc.begin());
            const int32_t nb = (int32_t)(std::lower_bound(nc.begin(), nc.end(), b) - nc.begin());
            const bool sa = std::binary_search(seeds.begin(), seeds.end(), na);
            const bool sb = std::binary_search(seeds.begin(), seeds.end(), nb);
            if (sa && !sb) add.push_back(nb);
            if (sb && !sa) add.push_back(na);
        }
        seeds.insert(seeds.end(), add.begin(), add.end());
        std::sort(seeds.begin() + 1, seeds.end());   // seeds[0] stays the first selected cell
    }
    const int tw = (cols + 7) / 8, th = (rows + 7) / 8, nt = tw * th;
    // links with a context-filled odd end need the top-down search's pending-extraction check
    bool tile = nt <= 16 * 1024 && !getenv("DMX_VSD_TOPDOWN") && g->nmamb == 0;
    int rc = DMX_OK;
    if (tile) {
        rc = prepare_uf(g);
        if (rc) return rc;
        rc = prepare_symmetry(g);
        if (rc) return rc;
        tile = g->symmetric == 1;
    }
    if (!tile) return visual_stepdepth_topdown(ctx, g, seeds, tw, th, out, sel);
    DevBuf<int32_t> d_seeds, d_level;
    HIPCHK(d_seeds.alloc(seeds.size()));
    HIPCHK(d_level.alloc((size_t)nt * 64));
    HIPCHK(hipMemcpyAsync(d_seeds.p, seeds.data(), seeds.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemsetAsync(d_level.p, 0xFF, (size_t)nt * 64 * 4, ctx->stream));
    std::vector<float> dummy(7);
    rc = vga_tile_impl(ctx, g, -1.0, 0, 0, 1, dummy.data(), false, nullptr, tw, th, d_seeds.p, (int)seeds.size(), d_level.p);
    if (rc == DMX_ERR_CAPACITY) return visual_stepdepth_topdown(ctx, g, seeds, tw, th, out, sel);
    if (rc) return rc;
    std::vector<int32_t> lv((size_t)nt * 64);
    HIPCHK(copy_sync(ctx->stream, lv.data(), d_level.p, lv.size() * 4, hipMemcpyDeviceToHost));
    for (int64_t k = 0; k < N; k++) {
        const int c = g->pm->node_cell[k];
        const int x = c / rows, y = c % rows;
        const int v = lv[(size_t)((((y >> 3) * tw + (x >> 3)) << 6) | ((y & 7) << 3) | (x & 7))];
        if (v >= 0) out[k] = (float)v;
    }
    for (int32_t k : seeds) out[k] = 0.0f;
    return DMX_OK;
}

int dmx_ctx_last_stepdepth(dmx_ctx* ctx, double* seconds, int64_t* expanders_popped, int64_t* cells_relaxed) {
    if (!ctx) return fail(DMX_ERR_ARG, "ctx is NULL");
    if (seconds) *seconds = ctx->last_sd_s;
    if (expanders_popped) *expanders_popped = ctx->last_sd_stats[0];
    if (cells_relaxed) *cells_relaxed = ctx->last_sd_stats[1];
    return DMX_OK;
}

int dmx_ctx_last_stepdepth_detail(dmx_ctx* ctx, int64_t* out4) {
    if (!ctx || !out4) return fail(DMX_ERR_ARG, "bad arguments");
    out4[0] = ctx->last_sd_mode;
    out4[1] = ctx->last_sd_stats[2];
    out4[2] = ctx->last_sd_extra[0];
    out4[3] = ctx->last_sd_extra[1];
    return DMX_OK;
}

// ---------------------------------------------------------------- .graph PointMap chunk
struct dmx_chunk {
    ParsedChunk pc;
};

int dmx_graph_from_runs(dmx_ctx* ctx, dmx_pointmap* pm, int64_t nnodes, const int32_t* bins, const int16_t* runs,
                        int64_t nruns, const uint8_t* gridconn, const float* attrs, dmx_graph** out) {
    if (!ctx || !pm || !out || nnodes < 0 || nruns < 0 || (nnodes && !bins) || (nruns && !runs))
        return fail(DMX_ERR_ARG, "bad arguments");
    HIPCHK(hipSetDevice(ctx->device));
    int rc = upload_pointmap(ctx, pm);
    if (rc) return rc;
    if (nnodes != pm->nnodes) return fail(DMX_ERR_ARG, "node count does not match the filled cells of the map");
    const int64_t N = nnodes;
    std::vector<int32_t> bn((size_t)std::max<int64_t>(N, 1) * 32), nr((size_t)std::max<int64_t>(N, 1));
    std::vector<uint16_t> bc((size_t)std::max<int64_t>(N, 1) * 32);
    std::vector<float> bd((size_t)std::max<int64_t>(N, 1) * 32);
    std::vector<int64_t> st((size_t)std::max<int64_t>(N, 1));
    int64_t acc = 0;
    for (int64_t k = 0; k < N; k++) {
        int s = 0;
        for (int b = 0; b < 32; b++) {
            const int32_t* r = bins + (k * 32 + b) * 4;
            bn[k * 32 + b] = r[3];
            bc[k * 32 + b] = (uint16_t)r[1];
            std::memcpy(&bd[k * 32 + b], &r[2], 4);
            s += r[3];
        }
        nr[k] = s;
        st[k] = acc;
        acc += s;
    }
    if (acc != nruns) return fail(DMX_ERR_ARG, "bins do not account for the runs");
    std::unique_ptr<dmx_graph> g(new dmx_graph());
    g->ctx = ctx; g->pm = pm; g->nnodes = N; g->node_begin = 0; g->node_end = N; g->nruns = nruns;
    inherit_merges(g.get());
    HIPCHK(g->pool.alloc(std::max<int64_t>(nruns, 1)));
    HIPCHK(g->node_run_start.alloc(std::max<int64_t>(N, 1)));
    HIPCHK(g->node_nruns.alloc(std::max<int64_t>(N, 1)));
    HIPCHK(g->bin_nruns.alloc(std::max<int64_t>(N, 1) * 32));
    HIPCHK(g->bin_count.alloc(std::max<int64_t>(N, 1) * 32));
    HIPCHK(g->bin_dist.alloc(std::max<int64_t>(N, 1) * 32));
    HIPCHK(g->attrs.alloc(std::max<int64_t>(N, 1) * 3));
    HIPCHK(g->gridconn.alloc(std::max<int64_t>(N, 1)));
    hipStream_t s = ctx->stream;
    if (nruns) HIPCHK(hipMemcpyAsync(g->pool.p, runs, nruns * 8, hipMemcpyHostToDevice, s));
    if (N) {
        HIPCHK(hipMemcpyAsync(g->node_run_start.p, st.data(), N * 8, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(g->node_nruns.p, nr.data(), N * 4, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(g->bin_nruns.p, bn.data(), N * 32 * 4, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(g->bin_count.p, bc.data(), N * 32 * 2, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(g->bin_dist.p, bd.data(), N * 32 * 4, hipMemcpyHostToDevice, s));
        if (attrs) HIPCHK(hipMemcpyAsync(g->attrs.p, attrs, N * 12, hipMemcpyHostToDevice, s));
        else HIPCHK(hipMemsetAsync(g->attrs.p, 0, N * 12, s));
        if (gridconn) HIPCHK(hipMemcpyAsync(g->gridconn.p, gridconn, N, hipMemcpyHostToDevice, s));
        else HIPCHK(hipMemsetAsync(g->gridconn.p, 0, N, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    *out = g.release();
    return DMX_OK;
}

int dmx_chunk_write(const dmx_pointmap* pm, int64_t nnodes, const int32_t* bins, const int16_t* runs, int64_t nruns,
                    const uint8_t* gridconn, int ncols, const char* const* names, const float* values,
                    const uint8_t* locked, const uint8_t* setmask, int displayed, int boundary, uint8_t* buf, int64_t cap,
                    int64_t* size) {
    if (!pm || !size || nnodes < 0 || ncols < 0 || (ncols && (!names || !values))) return fail(DMX_ERR_ARG, "bad arguments");
    std::vector<ChunkColumn> cols((size_t)ncols);
    for (int i = 0; i < ncols; i++) {
        cols[i].name = names[i];
        cols[i].locked = locked ? locked[i] != 0 : false;
        cols[i].values.assign(values + (size_t)i * nnodes, values + (size_t)(i + 1) * nnodes);
        if (setmask) cols[i].set.assign(setmask + (size_t)i * nnodes, setmask + (size_t)(i + 1) * nnodes);
    }
    std::vector<uint8_t> out;
    std::string err;
    if (write_pointmap_chunk(*pm->host, nnodes, bins, runs, nruns, gridconn, cols, displayed, boundary != 0, out, err))
        return fail(DMX_ERR_ARG, err);
    *size = (int64_t)out.size();
    if (buf) {
        if (cap < (int64_t)out.size()) return fail(DMX_ERR_ARG, "buffer too small");
        std::memcpy(buf, out.data(), out.size());
    }
    return DMX_OK;
}

int dmx_chunk_parse(const uint8_t* buf, int64_t size, dmx_chunk** out) {
    if (!buf || !out || size <= 0) return fail(DMX_ERR_ARG, "bad arguments");
    std::unique_ptr<dmx_chunk> c(new dmx_chunk());
    std::string err;
    if (read_pointmap_chunk(buf, (size_t)size, c->pc, err)) return fail(DMX_ERR_ARG, err);
    *out = c.release();
    return DMX_OK;
}

int dmx_chunk_free(dmx_chunk* c) {
    delete c;
    return DMX_OK;
}

int dmx_chunk_info(const dmx_chunk* c, int32_t* cols, int32_t* rows, double* spacing, double* bl, int64_t* nnodes,
                   int64_t* nruns, int32_t* ncols, int32_t* displayed_sorted, int64_t* bytes_used) {
    if (!c) return fail(DMX_ERR_ARG, "chunk is NULL");
    const ParsedChunk& p = c->pc;
    if (cols) *cols = p.cols;
    if (rows) *rows = p.rows;
    if (spacing) *spacing = p.spacing;
    if (bl) { bl[0] = p.blx; bl[1] = p.bly; }
    if (nnodes) *nnodes = (int64_t)p.gridconn.size();
    if (nruns) *nruns = (int64_t)p.runs.size() / 4;
    if (ncols) *ncols = (int32_t)p.columns.size();
    if (displayed_sorted) *displayed_sorted = p.displayed_sorted;
    if (bytes_used) *bytes_used = (int64_t)p.bytes_used;
    return DMX_OK;
}

int dmx_chunk_column(const dmx_chunk* c, int i, char* name, int name_cap, float* values, int* locked) {
    if (!c || i < 0 || i >= (int)c->pc.columns.size()) return fail(DMX_ERR_ARG, "bad column");
    const ChunkColumn& col = c->pc.columns[i];
    if (name && name_cap > 0) {
        const size_t n = std::min<size_t>(col.name.size(), (size_t)name_cap - 1);
        std::memcpy(name, col.name.data(), n);
        name[n] = 0;
    }
    if (values && !col.values.empty()) std::memcpy(values, col.values.data(), col.values.size() * 4);
    if (locked) *locked = col.locked ? 1 : 0;
    return DMX_OK;
}

int dmx_chunk_arrays(const dmx_chunk* c, int32_t* state, int32_t* bins, int16_t* runs, uint8_t* gridconn) {
    if (!c) return fail(DMX_ERR_ARG, "chunk is NULL");
    const ParsedChunk& p = c->pc;
    if (state) std::memcpy(state, p.state.data(), p.state.size() * 4);
    if (bins && !p.bins.empty()) std::memcpy(bins, p.bins.data(), p.bins.size() * 4);
    if (runs && !p.runs.empty()) std::memcpy(runs, p.runs.data(), p.runs.size() * 2);
    if (gridconn && !p.gridconn.empty()) std::memcpy(gridconn, p.gridconn.data(), p.gridconn.size());
    return DMX_OK;
}

int dmx_pointmap_set_state(dmx_pointmap* pm, const int32_t* state) {
    if (!pm || !state) return fail(DMX_ERR_ARG, "bad arguments");
    PointMapHost& h = *pm->host;
    h.restore_fill(state);
    pm->version++;
    return DMX_OK;
}

int dmx_chunk_load(dmx_ctx* ctx, const dmx_chunk* c, const double* region, dmx_pointmap** pm_out, dmx_graph** g_out) {
    if (!ctx || !c || !region || !pm_out || !g_out) return fail(DMX_ERR_ARG, "bad arguments");
    const ParsedChunk& p = c->pc;
    if (!p.processed) return fail(DMX_ERR_STATE, "the point map has no graph (run VISPREP -pm first)");
    Rect r{region[0], region[1], region[2], region[3]};
    std::unique_ptr<dmx_pointmap> pm(new dmx_pointmap());
    pm->host.reset(new PointMapHost(r, p.spacing, nullptr, 0));
    pm->host->load_state(p.cols, p.rows, p.spacing, Vec2{p.blx, p.bly}, p.state.data());
    const int64_t N = (int64_t)p.gridconn.size();
    std::vector<float> attrs((size_t)std::max<int64_t>(N, 1) * 3, 0.0f);
    const char* mk[3] = {"Connectivity", "Point First Moment", "Point Second Moment"};
    for (int j = 0; j < 3; j++)
        for (const auto& col : p.columns)
            if (col.name == mk[j] && (int64_t)col.values.size() == N)
                for (int64_t k = 0; k < N; k++) attrs[k * 3 + j] = col.values[k];
    dmx_graph* g = nullptr;
    int rc = dmx_graph_from_runs(ctx, pm.get(), N, p.bins.data(), p.runs.data(), (int64_t)p.runs.size() / 4,
                                 p.gridconn.data(), attrs.data(), &g);
    if (rc) return rc;
    std::unique_ptr<dmx_graph> gg(g);
    {
        std::vector<int32_t> per_cell, uniq;
        rc = normalize_merges(pm->host->cells(), p.merge_pairs.data(), (int64_t)p.merge_pairs.size() / 2, per_cell, uniq,
                              true);
        if (rc) return rc;
        pm->host->set_merge(std::move(per_cell));
    }
    inherit_merges(g);
    *pm_out = pm.release();
    *g_out = gg.release();
    return DMX_OK;
}

int dmx_pointmap_set_merges(dmx_pointmap* pm, const int32_t* cell_pairs, int64_t n) {
    if (!pm || n < 0 || (n && !cell_pairs)) return fail(DMX_ERR_ARG, "bad arguments");
    std::vector<int32_t> per_cell, uniq;
    if (int rc = normalize_merges(pm->host->cells(), cell_pairs, n, per_cell, uniq)) return rc;
    pm->host->set_merge(std::move(per_cell));
    return DMX_OK;
}

int dmx_graph_set_merges(dmx_graph* g, const int32_t* cell_pairs, int64_t n) {
    if (!g || n < 0 || (n && !cell_pairs)) return fail(DMX_ERR_ARG, "bad arguments");
    std::vector<int32_t> per_cell, uniq;
    if (int rc = normalize_merges(g->pm->host->cells(), cell_pairs, n, per_cell, uniq)) return rc;
    // the links belong to the points (Point::m_merge): the map gets them too, so a chunk written from it
    // saves them and a graph made from it again follows them
    g->pm->host->set_merge(std::move(per_cell));
    g->merges = std::move(uniq);
    g->merges_ready = false;
    if (g->merges.empty()) {   // prepare_merges returns early on no links: drop the previous links' device state
        g->nmamb = 0;
        g->d_mamb.reset();
        g->d_mpairs.reset();
        g->d_merge_cell.reset();
    }
    return DMX_OK;
}

int dmx_chunk_merges(const dmx_chunk* c, int32_t* cell_pairs, int64_t* n) {
    if (!c || !n) return fail(DMX_ERR_ARG, "bad arguments");
    std::vector<int32_t> per_cell, uniq;
    const ParsedChunk& p = c->pc;
    if (int rc = normalize_merges((int64_t)p.cols * p.rows, p.merge_pairs.data(), (int64_t)p.merge_pairs.size() / 2,
                                  per_cell, uniq, true))
        return rc;
    const int64_t m = (int64_t)uniq.size() / 2;
    if (cell_pairs) {
        if (*n < m) return fail(DMX_ERR_ARG, "buffer too small");
        std::memcpy(cell_pairs, uniq.data(), uniq.size() * 4);
    }
    *n = m;
    return DMX_OK;
}

int dmx_chunk_flags(const dmx_chunk* c, int* processed, int* boundary, int64_t* merges, int64_t* nrows) {
    if (!c) return fail(DMX_ERR_ARG, "chunk is NULL");
    if (processed) *processed = c->pc.processed ? 1 : 0;
    if (boundary) *boundary = c->pc.boundary ? 1 : 0;
    if (merges) *merges = c->pc.merges;
    if (nrows) *nrows = (int64_t)c->pc.row_keys.size();
    return DMX_OK;
}

int dmx_chunk_set_column(dmx_chunk* c, const char* name, const float* values, const uint8_t* setmask, int locked,
                         int make_displayed) {
    if (!c || !name || (!values && !c->pc.row_keys.empty())) return fail(DMX_ERR_ARG, "bad arguments");
    const int idx = chunk_set_column(c->pc, name, values, setmask, locked != 0);
    if (make_displayed) c->pc.displayed_phys = idx;
    return DMX_OK;
}

int dmx_chunk_set_displayed(dmx_chunk* c, int physical_column) {
    if (!c) return fail(DMX_ERR_ARG, "chunk is NULL");
    c->pc.displayed_phys = physical_column;
    return DMX_OK;
}

int dmx_chunk_set_name(dmx_chunk* c, const char* name) {
    if (!c || !name) return fail(DMX_ERR_ARG, "bad arguments");
    c->pc.name = name;
    return DMX_OK;
}

int dmx_chunk_select_cells(dmx_chunk* c, const int32_t* cells, int64_t n) {
    if (!c || (n && !cells)) return fail(DMX_ERR_ARG, "bad arguments");
    ParsedChunk& p = c->pc;
    const int64_t C = (int64_t)p.cols * p.rows;
    if ((int64_t)p.point_off.size() != C + 1) return fail(DMX_ERR_STATE, "chunk has no point records");
    for (int64_t i = 0; i < n; i++) {
        const int64_t cell = cells[i];
        if (cell < 0 || cell >= C) return fail(DMX_ERR_ARG, "cell outside the grid");
        if (!(p.state[cell] & CELL_FILLED)) continue;   // PointMap::setCurSel keeps filled cells only
        int32_t st;
        std::memcpy(&st, &p.points_raw[p.point_off[cell]], 4);
        st |= CELL_SELECTED;
        std::memcpy(&p.points_raw[p.point_off[cell]], &st, 4);
    }
    return DMX_OK;
}

int dmx_chunk_unmake(dmx_chunk* c, int remove_links) {
    if (!c) return fail(DMX_ERR_ARG, "chunk is NULL");
    std::string err;
    if (chunk_unmake(c->pc, remove_links != 0, err)) return fail(DMX_ERR_STATE, err);
    return DMX_OK;
}

int dmx_chunk_serialize(const dmx_chunk* c, uint8_t* buf, int64_t cap, int64_t* size) {
    if (!c || !size) return fail(DMX_ERR_ARG, "bad arguments");
    std::vector<uint8_t> out;
    std::string err;
    if (write_parsed_chunk(c->pc, out, err)) return fail(DMX_ERR_STATE, err);
    *size = (int64_t)out.size();
    if (buf) {
        if (cap < (int64_t)out.size()) return fail(DMX_ERR_ARG, "buffer too small");
        std::memcpy(buf, out.data(), out.size());
    }
    return DMX_OK;
}

// ---------------------------------------------------------------- .graph file (MetaGraph container)
struct dmx_graphfile {
    GraphFile gf;
    std::vector<double> lines;
};

int dmx_graphfile_read(const char* path, dmx_graphfile** out) {
    if (!path || !out) return fail(DMX_ERR_ARG, "bad arguments");
    FILE* f = fopen(path, "rb");
    if (!f) return fail(DMX_ERR_ARG, std::string("cannot open ") + path);
    std::vector<uint8_t> buf;
    uint8_t tmp[1 << 16];
    size_t k;
    while ((k = fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + k);
    fclose(f);
    std::unique_ptr<dmx_graphfile> g(new dmx_graphfile());
    std::string err;
    const int rc = read_graphfile(buf.data(), buf.size(), g->gf, err);
    if (rc == -2) return fail(DMX_ERR_UNSUPPORTED, err);
    if (rc) return fail(DMX_ERR_ARG, err);
    g->lines = graphfile_lines(g->gf);
    *out = g.release();
    return DMX_OK;
}

int dmx_graphfile_free(dmx_graphfile* g) {
    delete g;
    return DMX_OK;
}

int dmx_graphfile_write(const dmx_graphfile* g, const char* path) {
    if (!g || !path) return fail(DMX_ERR_ARG, "bad arguments");
    std::vector<uint8_t> out;
    std::string err;
    if (write_graphfile(g->gf, out, err)) return fail(DMX_ERR_STATE, err);
    FILE* f = fopen(path, "wb");
    if (!f) return fail(DMX_ERR_ARG, std::string("cannot write ") + path);
    const size_t w = fwrite(out.data(), 1, out.size(), f);
    fclose(f);
    if (w != out.size()) return fail(DMX_ERR_ARG, std::string("short write to ") + path);
    return DMX_OK;
}

int dmx_graphfile_info(const dmx_graphfile* g, int32_t* state, int32_t* view_class, double* region, int64_t* nlines,
                       int32_t* npointmaps, int32_t* displayed) {
    if (!g) return fail(DMX_ERR_ARG, "graph file is NULL");
    if (state) *state = g->gf.state;
    if (view_class) *view_class = g->gf.view_class;
    if (region) std::memcpy(region, g->gf.region, sizeof(g->gf.region));
    if (nlines) *nlines = (int64_t)g->lines.size() / 4;
    if (npointmaps) *npointmaps = (int32_t)g->gf.pointmaps.size();
    if (displayed) *displayed = g->gf.displayed_pointmap;
    return DMX_OK;
}

int dmx_graphfile_lines(const dmx_graphfile* g, double* lines) {
    if (!g || (!lines && !g->lines.empty())) return fail(DMX_ERR_ARG, "bad arguments");
    if (!g->lines.empty()) std::memcpy(lines, g->lines.data(), g->lines.size() * sizeof(double));
    return DMX_OK;
}

int dmx_graphfile_set_view(dmx_graphfile* g, int32_t state, int32_t view_class) {
    if (!g) return fail(DMX_ERR_ARG, "graph file is NULL");
    g->gf.state = state;
    g->gf.view_class = view_class;
    return DMX_OK;
}

int dmx_graphfile_pointmap(const dmx_graphfile* g, int i, const uint8_t** chunk, int64_t* size) {
    if (!g || !chunk || !size || i < 0 || i >= (int)g->gf.pointmaps.size()) return fail(DMX_ERR_ARG, "bad point map index");
    *chunk = g->gf.pointmaps[i].data();
    *size = (int64_t)g->gf.pointmaps[i].size();
    return DMX_OK;
}

int dmx_graphfile_put_pointmap(dmx_graphfile* g, int i, const uint8_t* chunk, int64_t size) {
    if (!g || !chunk || size <= 0 || i < -1 || i >= (int)g->gf.pointmaps.size()) return fail(DMX_ERR_ARG, "bad arguments");
    if (i < 0) {   // MetaGraph::addNewPointMap: appended and displayed
        g->gf.pointmaps.emplace_back(chunk, chunk + size);
        g->gf.displayed_pointmap = (int32_t)g->gf.pointmaps.size() - 1;
    } else {
        g->gf.pointmaps[i].assign(chunk, chunk + size);
    }
    return DMX_OK;
}

int dmx_graphfile_new_pointmap_name(const dmx_graphfile* g, char* name, int cap) {
    if (!g || !name || cap <= 0) return fail(DMX_ERR_ARG, "bad arguments");
    const std::string n = new_pointmap_name(g->gf, "VGA Map");
    if ((int)n.size() + 1 > cap) return fail(DMX_ERR_ARG, "buffer too small");
    std::memcpy(name, n.c_str(), n.size() + 1);
    return DMX_OK;
}

int32_t dmx_view_vga_top(int32_t view_class) { return view_vga_top(view_class); }

} // extern "C"
