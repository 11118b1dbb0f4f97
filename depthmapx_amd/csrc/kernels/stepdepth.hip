// stepdepth.hip -- VGA metric step depth (STEPDEPTH -sdt metric) on gfx950.
//
// Replaces VGAMetricDepth::run (salalib/vgamodules/vgametricdepth.cpp:23-92) with
// Node/Bin::extractMetric (salalib/ngraph.cpp:67-76, :330-345) and PointMap::blockedAdjacent
// (salalib/pointdata.cpp:1016-1068).
//
// The reference is a Dijkstra over a std::set<MetricTriple> ordered by (float dist, PixelRef) in
// which only "expanders" (the selected cells, BLOCKED cells and cells next to a BLOCKED cell)
// relax their visible cells.  Its results depend on the exact pop order (float sums, strict
// double-vs-float comparisons, set de-duplication that keeps the first lastpixel, cumulative
// angles overwritten on equal-distance updates), so this kernel keeps that order exactly:
//   * only expanders enter the priority queue; every other cell is final once every expander with
//     a smaller key has been processed (later candidates are never smaller), which is exactly
//     when the reference pops it;
//   * key(v) = (bits of the smallest distance ever queued for v) << 32 | PixelRef(v): the pop
//     order of the reference; a cell is "already popped" for expander u iff key(v) < key(u);
//   * one workgroup runs the sequential expander loop; the relaxation of each expander's runs
//     (tens of thousands of cells) is spread over its 1024 threads in <=128-cell chunks;
//   * the queue is an unsorted LDS window (parallel min per pop) refilled from an HBM overflow
//     list by distance windows.
#include <cstddef>

#include "common.hpp"

namespace dmx {

constexpr int SD_THREADS = 1024;
constexpr int SD_WIN = 4096;       // LDS queue window (u64 keys)
constexpr int SD_CHUNKQ = 4096;    // LDS queue of long-run chunks
constexpr int SD_CHUNK = 32;       // cells per chunk
constexpr int SD_BATCH = 8;        // cells whose state one lane loads at once
constexpr unsigned long long SD_INF = ~0ull;

// SDF_MERGE: the cell has a merge link (Point::m_merge): it is queued even when it does not expand,
// because its pop extracts the partner (vgametricdepth.cpp:68-83, vgametric.cpp:97-105,
// vgaangular.cpp:95-104, vgaangulardepth.cpp:57-67)
enum : uint8_t { SDF_FILLED = 1, SDF_EXPAND = 2, SDF_MERGE = 4 };

struct StepDepthParams {
    int cols, rows;
    const uint8_t* flags;          // [C] SDF_* per cell (x-major)
    const int32_t* cell_node;      // [C]
    const int64_t* node_run_start;
    const int32_t* node_nruns;
    const Run* pool;
    unsigned long long* key;       // [C] (min queued dist bits << 32) | PixelRef, SD_INF = never queued
    float* mdist;                  // [C] Point::m_dist (-1 initially)
    float* cum;                    // [C] Point::m_cumangle
    int32_t* lastpix;              // [C] lastpixel of the queued entry with the smallest key (-1: NoPixel)
    unsigned long long* over;      // HBM overflow list of queue keys
    int64_t over_cap;
    const int32_t* merge;          // [C] merge partner cell or -1 (nullptr: the map has no merge links)
    int* error;
    unsigned long long* stats;     // [0] expanders popped, [1] cells relaxed, [2] refills
};

__device__ __forceinline__ int pix_of(int x, int y) { return (x << 16) + (y & 0xffff); }   // pixelref.h:81
__device__ __forceinline__ unsigned long long sd_key(float d, int pix) {
    return ((unsigned long long)__float_as_uint(d) << 32) | (unsigned)pix;
}

struct SdShared {
    unsigned long long win[SD_WIN];
    int2 chunk[SD_CHUNKQ];          // (run index, first cell offset)
    unsigned long long red[SD_THREADS / 64];
    unsigned long long gmin;        // lower bound of the keys in the overflow list
    long long nover;                // entries in the overflow list
    int nwin, nchunk, cut_ok, ovf;  // ovf: the overflow list overflowed (sticky for the search)
    unsigned long long cur;         // key being popped
    float cut_w;                    // refill window width (distance units)
    unsigned long long keep;
    int idx, cnt;
};

__device__ __forceinline__ void sd_push(SdShared& S, const StepDepthParams& P, unsigned long long k) {
    // keys below the overflow bound go to the LDS window while it has room
    if (k < S.gmin) {
        const int pos = atomicAdd(&S.nwin, 1);
        if (pos < SD_WIN) { S.win[pos] = k; return; }
        atomicSub(&S.nwin, 1);
    }
    const long long o = atomicAdd((unsigned long long*)&S.nover, 1ull);
    if (o < P.over_cap) P.over[o] = k;
    else { atomicOr(P.error, KERR_FRONTIER); S.ovf = 1; }
    atomicMin(&S.gmin, k);
}

// PixelRef angle(a, b, c) / (pi/2) (pixelref.h:121-131) with a = (x, y), b = u, c = last.
__device__ __forceinline__ float sd_turn(int dx, int dy, int ux, int uy, int lastu) {
    if (lastu == -1) return 0.0f;
    const int lx = lastu >> 16, ly = lastu & 0xffff;
    const int ex = ux - lx, ey = uy - ly;
    return (float)(acos((double)(dx * ex + dy * ey) /
                        (sqrt((double)(dx * dx + dy * dy)) * sqrt((double)(ex * ex + ey * ey)) + 1e-12)) /
                   (3.14159265358979323846 * 0.5));
}

// Relax cell (x, y) from expander u: Bin::extractMetric (ngraph.cpp:330-345), or with ANG
// Bin::extractAngular (ngraph.cpp:348-366): the key is the cumulative angle, the update test
// here.angle + ang < cumangle (floats), and a cell reached with angle 0 expands too
// (Node::extractAngular expands when curs.angle == 0, ngraph.cpp:78-85).
template <bool ANG>
__device__ __forceinline__ void sd_relax(SdShared& S, const StepDepthParams& P, int64_t c, int x, int y, uint8_t f,
                                         unsigned long long kv, float mv, int ux, int uy, float du, float cumu,
                                         int lastu, unsigned long long ku, unsigned& relaxed) {
    if (!(f & SDF_FILLED)) return;        // diagonal-gap cells never resolve (p.filled() check)
    if (kv < ku) return;                  // already popped: m_misc == ~0
    // merge-linked cells carry explicit marks (lastpix -3 popped, -2 merged): with angular ties a cell
    // may be popped before u with a larger key, and a merged partner keeps the key of its link's pop
    if ((f & SDF_MERGE) && P.lastpix[c] <= -2) return;
    relaxed++;
    if (ANG) {
        const float cv = mv;              // P.cum[c]
        if (cv != -1.0f && !(du < cv)) return;   // ang >= 0 (or NaN): du + ang < cv cannot hold
        const float ang = sd_turn(x - ux, y - uy, ux, uy, lastu);
        if (cv == -1.0f || du + ang < cv) {
            const float nv = cumu + ang;
            P.cum[c] = nv;
            const unsigned long long nk = sd_key(nv, pix_of(x, y));
            if (nk < kv) {
                P.key[c] = nk;
                P.lastpix[c] = pix_of(ux, uy);
                if ((f & (SDF_EXPAND | SDF_MERGE)) || nv == 0.0f) sd_push(S, P, nk);
            }
        }
        return;
    }
    const int dx = x - ux, dy = y - uy;
    const double dd = sqrt((double)(dx * dx + dy * dy));
    const float md = mv;                  // P.mdist[c]
    if (md == -1.0f || (double)du + dd < (double)md) {
        const float nd = du + (float)dd;
        P.mdist[c] = nd;
        P.cum[c] = cumu + sd_turn(dx, dy, ux, uy, lastu);
        const unsigned long long nk = sd_key(nd, pix_of(x, y));
        if (nk < kv) {                    // a new smallest entry: it carries this lastpixel
            P.key[c] = nk;
            P.lastpix[c] = pix_of(ux, uy);
            if (f & (SDF_EXPAND | SDF_MERGE)) sd_push(S, P, nk);
        }
    }
}

// Cells [i0, i1) of run ru relaxed from expander u.  The cells of one expander's runs are distinct
// (every visible cell sits in one bin; diagonal gap cells lie on that bin's own diagonal), so the
// per-cell state of a batch of SD_BATCH cells is loaded up front -- up to 3*SD_BATCH independent
// loads in flight per lane instead of three dependent round trips per cell.
template <bool ANG>
__device__ __forceinline__ void sd_relax_span(SdShared& S, const StepDepthParams& P, const Run& ru, int i0, int i1,
                                              int ux, int uy, float du, float cumu, int lastu,
                                              unsigned long long ku, unsigned& relaxed) {
    const int dxs = (ru.x1 > ru.x0) ? 1 : 0;
    const int dys = (ru.y0 == ru.y1) ? 0 : ((ru.x0 == ru.x1) ? 1 : ((ru.y1 > ru.y0) ? 1 : -1));
    const float* mvp = ANG ? P.cum : P.mdist;
    for (int b = i0; b < i1; b += SD_BATCH) {
        const int n = min(SD_BATCH, i1 - b);
        uint8_t f[SD_BATCH];
        unsigned long long kv[SD_BATCH];
        float mv[SD_BATCH];
#pragma unroll
        for (int j = 0; j < SD_BATCH; j++) {
            if (j < n) {
                const int64_t c = (int64_t)(ru.x0 + (b + j) * dxs) * P.rows + (ru.y0 + (b + j) * dys);
                f[j] = P.flags[c];
                kv[j] = P.key[c];
                mv[j] = mvp[c];
            }
        }
#pragma unroll
        for (int j = 0; j < SD_BATCH; j++) {
            if (j < n) {
                const int x = ru.x0 + (b + j) * dxs, y = ru.y0 + (b + j) * dys;
                sd_relax<ANG>(S, P, (int64_t)x * P.rows + y, x, y, f[j], kv[j], mv[j], ux, uy, du, cumu, lastu, ku,
                              relaxed);
            }
        }
    }
}

// Relax every cell of a node's runs from u = (ux, uy) (Node::extractMetric / extractAngular): runs up
// to SD_CHUNK cells by their thread, longer tails through the LDS chunk queue (S.nchunk must be 0).
// A cell is "already popped" for u iff its key is below ku.
template <bool ANG>
__device__ void sd_relax_node(SdShared& S, const StepDepthParams& P, int node, int ux, int uy, float du, float cumu,
                              int lastu, unsigned long long ku, unsigned& relaxed) {
    const int tid = threadIdx.x;
    const int64_t rs = P.node_run_start[node];
    const int nr = P.node_nruns[node];
    for (int r = tid; r < nr; r += SD_THREADS) {
        const Run ru = P.pool[rs + r];
        const int len = max(ru.x1 - ru.x0, max(ru.y1 - ru.y0, ru.y0 - ru.y1)) + 1;
        sd_relax_span<ANG>(S, P, ru, 0, min(len, SD_CHUNK), ux, uy, du, cumu, lastu, ku, relaxed);
        for (int o = SD_CHUNK; o < len; o += SD_CHUNK) {
            const int q = atomicAdd(&S.nchunk, 1);
            if (q < SD_CHUNKQ) S.chunk[q] = make_int2(r, o);
            else sd_relax_span<ANG>(S, P, ru, o, min(len, o + SD_CHUNK), ux, uy, du, cumu, lastu, ku, relaxed);
        }
    }
    __syncthreads();
    const int nch = min(S.nchunk, SD_CHUNKQ);
    for (int j = tid; j < nch; j += SD_THREADS) {
        const int2 ch = S.chunk[j];
        const Run ru = P.pool[rs + ch.x];
        const int len = max(ru.x1 - ru.x0, max(ru.y1 - ru.y0, ru.y0 - ru.y1)) + 1;
        sd_relax_span<ANG>(S, P, ru, ch.y, min(len, ch.y + SD_CHUNK), ux, uy, du, cumu, lastu, ku, relaxed);
    }
    __syncthreads();
}

// The search of one workgroup from the nsel selected cells (all at distance 0).  rlim >= 0 stops it
// at the first pop with dist * spacing > rlim (VGAMetric's radius, vgametric.cpp:86-88): later
// pops can only resolve cells beyond the radius.
template <bool ANG>
__device__ void sd_run(SdShared& S, const StepDepthParams& P, const int32_t* sel, int nsel, double spacing,
                       double rlim, unsigned long long& popped, unsigned long long& refills, unsigned& relaxed) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    unsigned long long& s_keep = S.keep;
    int& s_idx = S.idx;
    int& s_cnt = S.cnt;
    if (tid == 0) {
        S.nwin = 0; S.nchunk = 0; S.gmin = SD_INF; S.nover = 0; S.cut_w = 4.0f; S.ovf = 0;
    }
    __syncthreads();
    // the selected cells enter at distance 0 (vgametricdepth.cpp:45-47)
    for (int i = tid; i < nsel; i += SD_THREADS) {
        const int c = sel[i];
        const unsigned long long k = sd_key(0.0f, pix_of(c / P.rows, c % P.rows));
        P.key[c] = k;
        if (ANG) P.cum[c] = 0.0f;         // m_cumangle of the selected cells (vgaangulardepth.cpp:39-42)
        sd_push(S, P, k);
    }
    __syncthreads();
    for (;;) {
        // ---- parallel min of the window (keys are unique)
        unsigned long long m = SD_INF;
        const int nw = min(S.nwin, SD_WIN);
        for (int i = tid; i < nw; i += SD_THREADS) m = min(m, S.win[i]);
        for (int off = 32; off >= 1; off >>= 1) m = min(m, (unsigned long long)__shfl_xor(m, off));
        if (lane == 0) S.red[wave] = m;
        __syncthreads();
        if (tid == 0) {
            unsigned long long mm = SD_INF;
            for (int w = 0; w < SD_THREADS / 64; w++) mm = min(mm, S.red[w]);
            S.cur = mm;
        }
        __syncthreads();
        const unsigned long long ku = S.cur;
        if (S.ovf) break;   // the overflow list overflowed: the caller re-runs this search
        if (ku == SD_INF || ku >= S.gmin) {
            if (S.nover == 0 && ku == SD_INF) break;
            // ---- refill: flush the window into the overflow list, then take back the smallest keys
            refills++;
            for (int i = tid; i < nw; i += SD_THREADS) {
                const long long o = atomicAdd((unsigned long long*)&S.nover, 1ull);
                if (o < P.over_cap) P.over[o] = S.win[i];
                else { atomicOr(P.error, KERR_FRONTIER); S.ovf = 1; }
                atomicMin(&S.gmin, S.win[i]);
            }
            __syncthreads();
            if (tid == 0) S.nwin = 0;
            const long long no = min(S.nover, P.over_cap);
            const unsigned long long g0 = S.gmin;
            unsigned long long cut;
            for (;;) {
                const float d0 = __uint_as_float((unsigned)(g0 >> 32));
                cut = max(sd_key(d0 + S.cut_w, 0), g0 + 1ull);
                int cnt = 0;
                for (long long i = tid; i < no; i += SD_THREADS) cnt += (P.over[i] < cut) ? 1 : 0;
                for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off);
                if (tid == 0) s_cnt = 0;
                __syncthreads();
                if (lane == 0) atomicAdd(&s_cnt, cnt);
                __syncthreads();
                const int total = s_cnt;
                __syncthreads();
                if (total <= SD_WIN || cut == g0 + 1ull) {
                    if (tid == 0 && total < SD_WIN / 8) S.cut_w *= 2.0f;
                    break;
                }
                if (tid == 0) S.cut_w *= 0.5f;
                __syncthreads();
            }
            // move valid keys below cut into the window, compact the valid rest in place
            if (tid == 0) { s_keep = 0; S.gmin = SD_INF; }
            __syncthreads();
            for (long long base = 0; base < no; base += SD_THREADS) {
                const long long i = base + tid;
                const unsigned long long k = (i < no) ? P.over[i] : SD_INF;
                bool valid = false;
                if (i < no) {
                    const int px = (int)((k >> 16) & 0xffff), py = (int)(k & 0xffff);
                    valid = P.key[(int64_t)px * P.rows + py] == k;
                }
                const bool in = valid && k < cut;
                const bool keep = valid && !in;
                if (in) S.win[atomicAdd(&S.nwin, 1)] = k;
                const unsigned long long km = __ballot(keep);
                unsigned long long kb = 0;
                if (lane == 0 && km) kb = atomicAdd(&s_keep, (unsigned long long)__popcll(km));
                kb = __shfl(kb, 0);
                __syncthreads();   // this block of P.over is read before it is overwritten
                if (keep) {
                    P.over[kb + __popcll(km & ((1ull << lane) - 1ull))] = k;
                    atomicMin(&S.gmin, k);
                }
                __syncthreads();
            }
            if (tid == 0) S.nover = (long long)s_keep;
            __syncthreads();
            continue;
        }
        // ---- pop ku: find its slot, move the last key into it
        for (int i = tid; i < nw; i += SD_THREADS)
            if (S.win[i] == ku) s_idx = i;
        __syncthreads();
        if (tid == 0) {
            S.win[s_idx] = S.win[nw - 1];
            S.nwin = nw - 1;
            S.nchunk = 0;
        }
        __syncthreads();
        const int ux = (int)((ku >> 16) & 0xffff), uy = (int)(ku & 0xffff);
        const int64_t uc = (int64_t)ux * P.rows + uy;
        if (P.key[uc] != ku) continue;    // stale: the cell was queued again with a smaller key
        const float du = __uint_as_float((unsigned)(ku >> 32));
        if (rlim >= 0.0 && (ANG ? (double)du : (double)du * spacing) > rlim) break;   // uniform (S.cur)
        popped++;
        const float cumu = P.cum[uc];
        const int lastu = P.lastpix[uc];
        // ---- relax: Node::extractMetric / extractAngular expand at distance (angle) 0, at BLOCKED and
        // at blocked-adjacent cells (ngraph.cpp:67-85); only merge-linked cells are queued otherwise
        if ((P.flags[uc] & SDF_EXPAND) || du == 0.0f)
            sd_relax_node<ANG>(S, P, P.cell_node[uc], ux, uy, du, cumu, lastu, ku, relaxed);
        // ---- merge pixel neither popped nor merged yet: it takes u's cumulative angle and is extracted
        // now from (here.dist, merge pixel, NoPixel), then counts as done (vgametricdepth.cpp:68-83,
        // vgaangulardepth.cpp:57-67).  Marks (lastpix): -3 = a merge-linked cell popped, -2 = merged.
        // The merged cell's key becomes ku (the step-depth rows read u's distance); VGAMetric /
        // VGAAngular do not count it (vgametric.cpp:97-110, vgaangular.cpp:95-106).  Keys cannot tell
        // "popped" here: an angular relaxation at equal angle queues a smaller PixelRef after u.
        if (P.merge && (P.flags[uc] & SDF_MERGE)) {
            const int m2 = P.merge[uc];
            const bool take = P.lastpix[m2] > -2;
            __syncthreads();   // every lane has read the marks
            if (tid == 0) {
                P.lastpix[uc] = -3;
                if (take) {
                    P.key[m2] = ku;
                    P.cum[m2] = cumu;
                    P.lastpix[m2] = -2;
                    S.nchunk = 0;
                }
            }
            __syncthreads();
            if (take && ((P.flags[m2] & SDF_EXPAND) || du == 0.0f))
                sd_relax_node<ANG>(S, P, P.cell_node[m2], m2 / P.rows, m2 % P.rows, du, cumu, -1, ku, relaxed);
        }
    }
    __syncthreads();
}

template <bool ANG>
__global__ void __launch_bounds__(SD_THREADS) stepdepth_kernel(StepDepthParams P, const int32_t* sel, int nsel) {
    __shared__ SdShared S;
    const int tid = threadIdx.x, lane = tid & 63;
    unsigned long long popped = 0, refills = 0;
    unsigned relaxed = 0;
    sd_run<ANG>(S, P, sel, nsel, 1.0, -1.0, popped, refills, relaxed);
    unsigned long long rl = relaxed;
    for (int off = 32; off >= 1; off >>= 1) rl += __shfl_xor(rl, off);
    if (lane == 0) atomicAdd(&P.stats[1], rl);
    if (tid == 0) { P.stats[0] = popped; P.stats[2] = refills; }
}

// ---------------------------------------------------------------- batched metric step depth
// The serial loop above pops one expander at a time.  Every relaxation adds dist(u, v) >= 1 grid
// unit, so no expander whose key lies below dmin + 1 (dmin = the smallest live key) can still be
// improved by any other live expander: all of them are final, and they form one batch whose
// relaxations run over the whole GPU.  What the batch must still reproduce is the reference's
// order-dependent fold of the batch's relaxations of one cell v (Bin::extractMetric,
// ngraph.cpp:330-345, applied in pop order):
//     if (md == -1 || du + dd < md) { md = du + float(dd); cum = cum_u + turn; set entry (md, v, u) }
// Let s = du + dd (double) and f = du + float(dd) (float): |f - s| <= 2^-23 s.  If the smallest
// candidate s_m has no rival within W = 2^-20 s_m, the fold's outcome is exactly "apply m's update
// to the pre-batch state": an earlier success j leaves md = f_j > s_m, so m still succeeds, and after
// m every later candidate has s > f_m.  Candidates with s > md0 (1 + 2^-20) can then never succeed
// and are skipped.  Cells with a near rival ("ambiguous": exact ties on the grid are common) are
// folded sequentially in pop order from the list of all their batch relaxers.  A batch is the
// contiguous key range below the threshold, so batches run in the reference's pop order.
// Kernels per batch: select -> relax<1> (min s) -> relax<2> (rivals) -> apply -> relax<3> (ambiguous
// relaxer lists) -> fold -> finish.  Any capacity overflow raises ctl.error and the host re-runs the
// search with the serial kernel.
constexpr int SDB_THREADS = 256;
constexpr int SDB_UNIT = 256;          // runs of one expander per work unit (one workgroup)
constexpr int SDB_FOLD_CAP = 2048;     // relaxers of one ambiguous cell in one batch

struct SdbExp {
    int64_t rs;                 // first run of the expander's node in the pool
    unsigned long long ku;      // the expander's key (pop order)
    float du, cumu;
    int ux, uy, lastu, nr, ubase, pad;
};

struct SdbCtl {
    unsigned long long gcur, gnext;   // smallest live expander key: this batch / the next one
    unsigned nb, nunits, ntouch, namb, nent, done, error, batches;
    unsigned long long relaxed, improved, ambiguous, popped;
};

struct SdbParams {
    int rows;
    int64_t E;
    const uint8_t* flags;
    const int32_t* cell_node;
    const int64_t* node_run_start;
    const int32_t* node_nruns;
    const Run* pool;
    unsigned long long* key;
    float* mdist;
    float* cum;
    int32_t* lastpix;
    const int32_t* ex_cells;      // [E] expander cells (BLOCKED, blocked-adjacent, selected)
    uint8_t* ex_done;             // [E] popped
    SdbExp* bq;                   // [E] batch
    int32_t* uown;                // [units] batch index of each work unit
    unsigned long long* best;     // [C] smallest candidate s of the batch (double bits), ~0 = none
    unsigned* nnear;              // [C] candidates within W of best
    int32_t* win;                 // [C] batch index of the candidate at best
    int32_t* ambid;               // [C] ambiguous-cell index, -1
    int32_t* touch;               // [C] cells with a candidate this batch
    int32_t* amb;                 // [amb_cap] ambiguous cells
    int2* ent;                    // [ent_cap] (ambiguous index, batch index)
    int32_t* ahead;               // [amb_cap] last entry of each ambiguous cell's relaxer list (-1: none)
    int32_t* enext;               // [ent_cap] previous entry of the same ambiguous cell (-1: none)
    unsigned ent_cap, amb_cap;
    SdbCtl* ctl;
};

__device__ __forceinline__ double sdb_w(double s) { return s * 0x1p-20; }

// Append `want` lanes of the wave to a list: one atomic per wave.
__device__ __forceinline__ unsigned sdb_wave_append(unsigned* counter, bool want) {
    const unsigned long long m = __ballot(want);
    if (!m) return 0;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)m) - 1;
    unsigned base = 0;
    if (lane == leader) base = atomicAdd(counter, (unsigned)__popcll(m));
    base = __shfl(base, leader);
    return base + (unsigned)__popcll(m & ((1ull << lane) - 1ull));
}

__global__ void sdb_select_kernel(SdbParams P) {
    SdbCtl& C = *P.ctl;
    const unsigned long long g = C.gcur;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g == SD_INF || C.error) return;
    bool take = false;
    int c = 0;
    unsigned long long k = SD_INF;
    if (e < P.E && !P.ex_done[e]) {
        c = P.ex_cells[e];
        k = P.key[c];
        if (k != SD_INF) {
            const double lim = (double)__uint_as_float((unsigned)(g >> 32)) + 1.0;
            if ((double)__uint_as_float((unsigned)(k >> 32)) < lim - lim * 0x1p-18) take = true;
            else atomicMin(&C.gnext, k);
        }
    }
    const unsigned bi = sdb_wave_append(&C.nb, take);
    if (!take) return;
    P.ex_done[e] = 1;
    const int node = P.cell_node[c];
    SdbExp X;
    X.rs = P.node_run_start[node];
    X.nr = P.node_nruns[node];
    X.ku = k;
    X.du = __uint_as_float((unsigned)(k >> 32));
    X.cumu = P.cum[c];
    X.ux = c / P.rows;
    X.uy = c % P.rows;
    X.lastu = P.lastpix[c];
    const int nu = (X.nr + SDB_UNIT - 1) / SDB_UNIT;
    X.ubase = (int)atomicAdd(&C.nunits, (unsigned)nu);
    X.pad = 0;
    P.bq[bi] = X;
    for (int j = 0; j < nu; j++) P.uown[X.ubase + j] = (int)bi;
}

// PH 1: candidate minimum per cell; PH 2: rivals within W of it; PH 3: relaxer lists of the
// ambiguous cells.  One workgroup per (expander, <= SDB_UNIT runs); the unit's cells are spread over
// the threads through an LDS prefix sum of the run lengths.
template <int PH>
__global__ void __launch_bounds__(SDB_THREADS) sdb_relax_kernel(SdbParams P) {
    __shared__ Run runs[SDB_UNIT];
    __shared__ int off[SDB_UNIT + 1];
    __shared__ int wsum[SDB_THREADS / 64];
    SdbCtl& C = *P.ctl;
    if (C.error) return;
    if (PH == 3 && C.namb == 0) return;
    const unsigned nunits = C.nunits;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    unsigned long long relaxed = 0;
    for (unsigned u = blockIdx.x; u < nunits; u += gridDim.x) {
        const int b = P.uown[u];
        const SdbExp X = P.bq[b];
        const int r0 = ((int)u - X.ubase) * SDB_UNIT;
        const int nr = min(SDB_UNIT, X.nr - r0);
        int len = 0;
        if (t < nr) {
            const Run ru = P.pool[X.rs + r0 + t];
            runs[t] = ru;
            len = max(ru.x1 - ru.x0, max(ru.y1 - ru.y0, ru.y0 - ru.y1)) + 1;
        }
        int inc = len;   // inclusive wave scan, then the wave totals
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(inc, o);
            if (lane >= o) inc += v;
        }
        if (lane == 63) wsum[wave] = inc;
        __syncthreads();
        int base = 0;
        for (int w = 0; w < wave; w++) base += wsum[w];
        off[t + 1] = base + inc;
        if (t == 0) off[0] = 0;
        __syncthreads();
        const int T = off[nr];
        for (int i = t; i < T; i += SDB_THREADS) {
            int lo = 0, hi = nr - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (off[mid] <= i) lo = mid;
                else hi = mid - 1;
            }
            const Run ru = runs[lo];
            const int k = i - off[lo];
            const int dxs = (ru.x1 > ru.x0) ? 1 : 0;
            const int dys = (ru.y0 == ru.y1) ? 0 : ((ru.x0 == ru.x1) ? 1 : ((ru.y1 > ru.y0) ? 1 : -1));
            const int x = ru.x0 + k * dxs, y = ru.y0 + k * dys;
            const int64_t c = (int64_t)x * P.rows + y;
            bool cand = false;
            double s = 0.0;
            if (P.flags[c] & SDF_FILLED) {
                if (P.key[c] >= X.ku) {   // not popped before u (m_misc == 0)
                    const int dx = x - X.ux, dy = y - X.uy;
                    s = (double)X.du + sqrt((double)(dx * dx + dy * dy));
                    if (PH == 3) {
                        cand = P.ambid[c] >= 0;
                    } else {
                        const float md = P.mdist[c];
                        cand = md == -1.0f || s <= (double)md + sdb_w((double)md);
                    }
                    if (PH == 1) relaxed++;
                }
            }
            if (PH == 1) {
                bool first = false;
                if (cand) first = atomicMin(&P.best[c], (unsigned long long)__double_as_longlong(s)) == SD_INF;
                const unsigned pos = sdb_wave_append(&C.ntouch, first);
                if (first) P.touch[pos] = (int32_t)c;
            } else if (PH == 2) {
                if (cand) {
                    const double bs = __longlong_as_double((long long)P.best[c]);
                    if (s <= bs + sdb_w(bs)) {
                        atomicAdd(&P.nnear[c], 1u);
                        if (s == bs) P.win[c] = b;
                    }
                }
            } else {
                const unsigned pos = sdb_wave_append(&C.nent, cand);
                if (cand) {
                    if (pos < P.ent_cap) {
                        const int a = P.ambid[c];
                        P.ent[pos] = make_int2(a, b);
                        P.enext[pos] = atomicExch(&P.ahead[a], (int)pos);   // per-cell list: O(entries) fold
                    } else {
                        C.error = 1;
                    }
                }
            }
        }
        __syncthreads();
    }
    if (PH == 1) {
        for (int o = 32; o >= 1; o >>= 1) relaxed += __shfl_xor(relaxed, o);
        if (lane == 0 && relaxed) atomicAdd(&C.relaxed, relaxed);
    }
}

// One relaxation of cell c = (x, y) from batch expander X, in the reference's sequential form
// (sd_relax without the popped test, which the relax kernels already applied).
__device__ __forceinline__ void sdb_update(const SdbParams& P, SdbCtl& C, int64_t c, int x, int y, uint8_t f,
                                           const SdbExp& X) {
    const int dx = x - X.ux, dy = y - X.uy;
    const double dd = sqrt((double)(dx * dx + dy * dy));
    const float md = P.mdist[c];
    if (md == -1.0f || (double)X.du + dd < (double)md) {
        const float nd = X.du + (float)dd;
        P.mdist[c] = nd;
        P.cum[c] = X.cumu + sd_turn(dx, dy, X.ux, X.uy, X.lastu);
        const unsigned long long nk = sd_key(nd, pix_of(x, y));
        if (nk < P.key[c]) {
            P.key[c] = nk;
            P.lastpix[c] = pix_of(X.ux, X.uy);
            if (f & SDF_EXPAND) atomicMin(&C.gnext, nk);
        }
    }
}

__global__ void sdb_apply_kernel(SdbParams P) {
    SdbCtl& C = *P.ctl;
    if (C.error) return;
    const unsigned n = C.ntouch;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int c = P.touch[i];
        const unsigned nn = P.nnear[c];
        P.best[c] = SD_INF;
        P.nnear[c] = 0u;
        if (nn == 1u) {
            const SdbExp X = P.bq[P.win[c]];
            sdb_update(P, C, c, c / P.rows, c % P.rows, P.flags[c], X);
        } else {
            const unsigned a = atomicAdd(&C.namb, 1u);
            if (a < P.amb_cap) {
                P.amb[a] = c;
                P.ambid[c] = (int)a;
            } else {
                C.error = 1;
            }
        }
    }
}

// Sequential fold of each ambiguous cell over all its batch relaxers in pop (key) order.
__global__ void __launch_bounds__(SDB_THREADS) sdb_fold_kernel(SdbParams P) {
    __shared__ int lst[SDB_FOLD_CAP];
    SdbCtl& C = *P.ctl;
    if (C.error) return;
    const unsigned na = min(C.namb, P.amb_cap);
    // one thread per ambiguous cell walks its relaxer list (built by sdb_relax_kernel<3>), so a batch
    // costs O(entries) rather than a scan of every entry per ambiguous cell
    for (unsigned a = blockIdx.x * blockDim.x + threadIdx.x; a < na; a += gridDim.x * blockDim.x) {
        int n = 0;
        bool over = false;
        // relaxers in pop order: insertion sort by the relaxer's key while walking the list
        int buf[32];
        int* lp = buf;
        for (int e = P.ahead[a]; e >= 0; e = P.enext[e]) {
            if (n == 32) { over = true; break; }
            const int v = P.ent[e].y;
            const unsigned long long kv = P.bq[v].ku;
            int j = n - 1;
            while (j >= 0 && P.bq[lp[j]].ku > kv) { lp[j + 1] = lp[j]; j--; }
            lp[j + 1] = v;
            n++;
        }
        if (over) continue;   // long lists: the block pass below
        const int c = P.amb[a];
        const uint8_t f = P.flags[c];
        for (int i = 0; i < n; i++) sdb_update(P, C, c, c / P.rows, c % P.rows, f, P.bq[lp[i]]);
        P.ambid[c] = -1;
        P.ahead[a] = -1;
    }
    // cells with more than 32 relaxers: one block per cell, the list gathered into LDS, folded by thread
    // 0.  Which pass folds a cell depends only on its list length (the thread pass clears the head of
    // the short lists it folds, at any time relative to this loop, and never touches a long one).
    for (unsigned a = blockIdx.x; a < na; a += gridDim.x) {
        if (threadIdx.x == 0) {
            const int h = P.ahead[a];
            int len = 0;
            for (int e = h; e >= 0 && len <= 32; e = P.enext[e]) len++;
            if (len <= 32) continue;
            int n = 0;
            for (int e = h; e >= 0; e = P.enext[e]) {
                if (n == SDB_FOLD_CAP) { C.error = 1; n = -1; break; }
                lst[n++] = P.ent[e].y;
            }
            if (n >= 0) {
                for (int i = 1; i < n; i++) {   // insertion sort by the relaxer's key (pop order)
                    const int v = lst[i];
                    const unsigned long long kv = P.bq[v].ku;
                    int j = i - 1;
                    while (j >= 0 && P.bq[lst[j]].ku > kv) { lst[j + 1] = lst[j]; j--; }
                    lst[j + 1] = v;
                }
                const int c = P.amb[a];
                const uint8_t f = P.flags[c];
                for (int i = 0; i < n; i++) sdb_update(P, C, c, c / P.rows, c % P.rows, f, P.bq[lst[i]]);
                P.ambid[c] = -1;
            }
            P.ahead[a] = -1;
        }
    }
}

// The selected cells enter at distance 0 (vgametricdepth.cpp:45-47).
__global__ void sdb_init_kernel(SdbParams P, const int32_t* sel, int nsel) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nsel) P.key[sel[i]] = sd_key(0.0f, pix_of(sel[i] / P.rows, sel[i] % P.rows));
}

__global__ void sdb_finish_kernel(SdbParams P) {
    SdbCtl& C = *P.ctl;
    if (C.nb) C.batches++;
    C.popped += C.nb;
    C.improved += C.ntouch;
    C.ambiguous += C.namb;
    C.gcur = C.gnext;
    C.gnext = SD_INF;
    C.nb = 0; C.nunits = 0; C.ntouch = 0; C.namb = 0; C.nent = 0;
    if (C.gcur == SD_INF || C.error) C.done = 1;
}

// ---------------------------------------------------------------- VGA metric (all sources)
// VGAMetric::run (salalib/vgamodules/vgametric.cpp:26-136): the search above from every source,
// one source per workgroup at a time (per-workgroup key / dist / angle arrays in HBM), followed by
// the reference's float totals, which are accumulated in pop order = ascending key order:
//   total_depth += float(dist * spacing), total_angle += cumangle,
//   euclid_depth += float(spacing * dist(cell, source)), total_nodes++.
// Ordering: the reached keys are bucketed by distance (VM_BUCKETS, counting sort through HBM), a
// window of whole buckets (<= VM_CAP keys) is bitonic-sorted in the LDS the search no longer needs,
// and wave 0 adds the terms lane by lane (readlane) -- the reference's sequential float chains.
constexpr int VM_BUCKETS = 1024;
constexpr int VM_CAP = 2 * SD_WIN;     // keys sorted at once: the search's window + chunk queue LDS

template <bool ANG>
__global__ void __launch_bounds__(SD_THREADS) vga_metric_kernel(StepDepthParams P0, int64_t C, const int32_t* node_cell,
                                                                int64_t sb, int64_t se, int gates_only, double spacing,
                                                                double radius, unsigned long long* comp_all,
                                                                unsigned long long* srt_all, int64_t nstride,
                                                                float* out, const int64_t* src_list,
                                                                int64_t* fail_list, int* fail_count) {
    __shared__ SdShared S;
    __shared__ int hoff[VM_BUCKETS + 1];
    __shared__ int cur[VM_BUCKETS];
    __shared__ int s_src, s_n, s_pos, s_wend;
    __shared__ unsigned s_maxd;
    static_assert(offsetof(SdShared, chunk) == SD_WIN * sizeof(unsigned long long), "window + chunk queue contiguous");
    unsigned long long* sk = S.win;   // VM_CAP keys (spans win and chunk)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t b = blockIdx.x;
    StepDepthParams P = P0;
    P.key = P0.key + b * C;
    P.mdist = P0.mdist + b * C;
    P.cum = P0.cum + b * C;
    P.lastpix = P0.lastpix + b * C;
    P.over = P0.over + b * P0.over_cap;
    unsigned long long* comp = comp_all + b * 2 * nstride;   // [2N]: compaction, then the sort of an oversize bucket
    unsigned long long* srt = srt_all + b * nstride;
    unsigned long long popped = 0, refills = 0;
    unsigned relaxed = 0;
    // sources sb + i, or src_list[i] on a re-run of the sources whose overflow list overflowed
    const int64_t nwork = src_list ? se : se - sb;
    for (int64_t i = blockIdx.x; i < nwork; i += gridDim.x) {
        const int64_t src = src_list ? src_list[i] : sb + i;
        constexpr int NO = ANG ? 3 : 4;
        float* o = out + src * NO;
        if (gates_only) {
            if (tid < NO) o[tid] = -1.0f;
            continue;
        }
        for (int64_t c = tid; c < C; c += SD_THREADS) {
            P.key[c] = SD_INF;
            P.mdist[c] = -1.0f;
            P.cum[c] = ANG ? -1.0f : 0.0f;
            P.lastpix[c] = -1;
        }
        if (tid == 0) { s_src = node_cell[src]; s_n = 0; s_pos = 0; s_maxd = 0u; }
        __syncthreads();
        sd_run<ANG>(S, P, &s_src, 1, spacing, radius, popped, refills, relaxed);
        __syncthreads();
        if (S.ovf) {   // this source only: re-run by the host with a larger list
            if (tid == 0) fail_list[atomicAdd(fail_count, 1)] = src;
            continue;
        }
        const int sx = s_src / P.rows, sy = s_src % P.rows;
        // reached cells within the radius: count and largest distance
        int n = 0;
        unsigned md = 0u;
        for (int64_t c = tid; c < C; c += SD_THREADS) {
            const unsigned long long k = P.key[c];
            if (k == SD_INF || (P.merge && P.lastpix[c] == -2)) continue;   // merged partners are not counted
            const float d = __uint_as_float((unsigned)(k >> 32));
            if (radius >= 0.0 && (ANG ? (double)d : (double)d * spacing) > radius) continue;
            n++;
            md = max(md, (unsigned)(k >> 32));   // non-negative floats order like their bits
        }
        for (int off = 32; off >= 1; off >>= 1) {
            n += __shfl_xor(n, off);
            md = max(md, (unsigned)__shfl_xor((int)md, off));
        }
        for (int i = tid; i < VM_BUCKETS; i += SD_THREADS) cur[i] = 0;
        if (lane == 0) { atomicAdd(&s_n, n); atomicMax(&s_maxd, md); }
        __syncthreads();
        const int nt = s_n;
        const float inv = (float)VM_BUCKETS / fmaxf(__uint_as_float(s_maxd), 1e-30f);
        // histogram + compaction (any order)
        for (int64_t c = tid; c < C; c += SD_THREADS) {
            const unsigned long long k = P.key[c];
            if (k == SD_INF || (P.merge && P.lastpix[c] == -2)) continue;
            const float d = __uint_as_float((unsigned)(k >> 32));
            if (radius >= 0.0 && (ANG ? (double)d : (double)d * spacing) > radius) continue;
            const int bk = min(VM_BUCKETS - 1, (int)(d * inv));
            atomicAdd(&cur[bk], 1);
            comp[atomicAdd(&s_pos, 1)] = k;
        }
        __syncthreads();
        if (tid == 0) {
            int acc = 0;
            for (int i = 0; i < VM_BUCKETS; i++) { hoff[i] = acc; acc += cur[i]; cur[i] = hoff[i]; }
            hoff[VM_BUCKETS] = acc;
        }
        __syncthreads();
        for (int i = tid; i < nt; i += SD_THREADS) {
            const unsigned long long k = comp[i];
            const int bk = min(VM_BUCKETS - 1, (int)(__uint_as_float((unsigned)(k >> 32)) * inv));
            srt[atomicAdd(&cur[bk], 1)] = k;
        }
        __syncthreads();
        // windows of whole buckets, sorted in LDS, summed in order by wave 0
        float td = 0.0f, ta = 0.0f, te = 0.0f;
        int bs = 0;
        while (bs < VM_BUCKETS) {
            if (tid == 0) {
                int be = bs + 1;
                while (be < VM_BUCKETS && hoff[be + 1] - hoff[bs] <= VM_CAP) be++;
                s_wend = be;
            }
            __syncthreads();
            const int be = s_wend;
            const int w0 = hoff[bs], m = hoff[be] - w0;
            // a window is whole buckets of <= VM_CAP keys, sorted in LDS; a single bucket above that
            // (e.g. every cell seen straight from the source sits at angle 0) is sorted in HBM scratch
            unsigned long long* arr = m > VM_CAP ? comp : sk;
            int p2 = 1;
            while (p2 < m) p2 <<= 1;
            for (int i = tid; i < p2; i += SD_THREADS) arr[i] = i < m ? srt[w0 + i] : SD_INF;
            __syncthreads();
            for (int k = 2; k <= p2; k <<= 1)
                for (int j = k >> 1; j > 0; j >>= 1) {
                    for (int i = tid; i < p2; i += SD_THREADS) {
                        const int ixj = i ^ j;
                        if (ixj > i) {
                            const unsigned long long a = arr[i], c2 = arr[ixj];
                            if ((a > c2) == ((i & k) == 0)) { arr[i] = c2; arr[ixj] = a; }
                        }
                    }
                    __syncthreads();
                }
            if (wave == 0) {
                for (int i0 = 0; i0 < m; i0 += 64) {
                    const int i = i0 + lane;
                    float t0 = 0.0f, t1 = 0.0f, t2 = 0.0f;
                    if (i < m) {
                        const unsigned long long k = arr[i];
                        const int x = (int)((k >> 16) & 0xffff), y = (int)(k & 0xffff);
                        const float d = __uint_as_float((unsigned)(k >> 32));
                        const int dx = x - sx, dy = y - sy;
                        t0 = (float)((double)d * spacing);
                        t1 = P.cum[(int64_t)x * P.rows + y];
                        t2 = (float)(spacing * sqrt((double)(dx * dx + dy * dy)));
                    }
                    const int cnt = min(64, m - i0);
                    for (int l = 0; l < cnt; l++) {
                        td += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t0), l));
                        ta += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t1), l));
                        te += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t2), l));
                    }
                }
            }
            __syncthreads();
            bs = be;
        }
        if (tid == 0) {
            if (ANG) {   // vgaangular.cpp:113-118 (nt >= 1: the source itself)
                o[0] = (float)((double)ta / (double)nt);
                o[1] = ta;
                o[2] = (float)nt;
            } else {
                o[0] = (float)((double)ta / (double)nt);
                o[1] = (float)((double)td / (double)nt);
                o[2] = (float)((double)te / (double)nt);
                o[3] = (float)nt;
            }
        }
        __syncthreads();
    }
    unsigned long long rl = relaxed;
    for (int off = 32; off >= 1; off >>= 1) rl += __shfl_xor(rl, off);
    if (lane == 0) atomicAdd(&P0.stats[1], rl);
    if (tid == 0) { atomicAdd(&P0.stats[0], popped); atomicAdd(&P0.stats[2], refills); }
}

// Attribute rows (vgametricdepth.cpp:54-61): float(spacing * dist), cumulative angle and, for a
// single selected cell, the straight-line distance.
__global__ void stepdepth_out_kernel(int rows, double spacing, const int32_t* node_cell, int64_t n,
                                     const unsigned long long* key, const float* cum, int single, int selx, int sely,
                                     float* out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const int c = node_cell[k];
    const unsigned long long kv = key[c];
    float* o = out + k * 3;
    if (kv == SD_INF) { o[0] = -1.0f; o[1] = -1.0f; o[2] = -1.0f; return; }
    const float d = __uint_as_float((unsigned)(kv >> 32));
    o[0] = cum[c];
    o[1] = (float)(spacing * (double)d);
    if (single) {
        const int dx = c / rows - selx, dy = c % rows - sely;
        o[2] = (float)(spacing * sqrt((double)(dx * dx + dy * dy)));
    } else {
        o[2] = -1.0f;
    }
}

} // namespace dmx
