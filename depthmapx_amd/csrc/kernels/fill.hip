// fill.hip -- VISPREP on the GPU: occluder rasterisation and the flood fill that precede makeGraph.
//
//   blockLines / blockLine   salalib/pointdata.cpp:296-357   every drawing line is appended to each
//   pixelateLineTouching     salalib/spacepix.cpp:144-214    cell it touches (tolerance 1e-10), the
//   Line::crop               genlib/p2dpoly.cpp:626-667      cells become BLOCKED, and each cell crops
//                                                            its copies to regionate(cell, 1e-10)
//   makePoints / expand      salalib/pointdata.cpp:402-514   8-neighbour flood fill from the seed
//
// Rasterisation: one thread per drawing line walks the line's columns (or rows) as the reference
// does and emits the touched cells; the per-cell line lists are placed by a count / exclusive-scan /
// scatter pass and sorted by line index (the reference appends lines in drawing order), then one
// thread per cell crops its copies in that order.  All geometry is the shared __host__ __device__
// code of host/geometry.hpp, IEEE double in the reference's operation order.
//
// Flood fill.  The reference fills with two stacks ("pflipper"): it pops the current layer from the
// back, and every expand that finds its neighbour unfilled and unblocked fills it and pushes it onto
// the next layer.  The FILLED set is plain reachability, but the EDGE bit is order dependent: expand
// only tests the occluders when the neighbour is still unfilled, so a cell is an edge iff it is
// BLOCKED or some blocked step leads to a neighbour not yet filled *at that moment*.  The kernels
// reproduce the exact order level by level:
//   - layer d is held in processing order; expand call (p, k) -- the p-th processed cell, direction
//     k -- precedes (p', k') iff p*8+k < p'*8+k';
//   - claim: every unblocked call on a cell unfilled at the start of the layer does
//     atomicMin(owner[c2], p*8+k); the minimum is the call that fills c2 in the reference;
//   - resolve: a blocked call (p, k) meets an unfilled neighbour iff owner[c2] > p*8+k (neighbours
//     filled before the layer started were filled by then, and owner is the fill time of the rest);
//   - push: the cells owned by p, in direction order, take consecutive push positions after an
//     exclusive scan over p; the next layer's processing order is the reverse of the push order,
//     because the reference pops from the back.
// Cells filled by an earlier fill call simply count as filled from the start.
#pragma once

namespace dmx {

constexpr int FILL_THREADS = 256;

// Grid geometry of the host model (PointMap::setGrid, pointdata.cpp:122-171).
struct FillGrid {
    int cols, rows;
    double spacing;
    double blx, bly;   // bottom-left cell centre (m_bottom_left)
    Rect region;       // the grid region (m_region), for PixelBase::pixelateLineTouching's normalScale
    int32_t fill_state = CELL_FILLED;   // Point::set's state for this fill: FILLED [| CONTEXTFILLED] (:434-441)
};

__device__ __forceinline__ Seg drawing_seg(const double* draw, int64_t k) {
    return make_seg(Vec2{draw[4 * k], draw[4 * k + 1]}, Vec2{draw[4 * k + 2], draw[4 * k + 3]});
}

// PixelBase::pixelateLineTouching(l, 1e-10) (spacepix.cpp:144-214): emit(cell index) for every
// touched cell inside the grid, in the reference's order.  Iterations whose column (row) lies off
// the grid emit nothing in the reference (PixelRef::encloses), so the loop skips them; for grids of
// at most 16000 cells a side the short casts of the reference are the identity on what remains.
template <class Emit>
__device__ void rasterise_line(const FillGrid& G, Seg l, Emit&& emit) {
    const double tol = 1e-10;
    const double rw = G.region.width(), rh = G.region.height();
    l.r.trx = rw ? (l.r.trx - G.region.blx) / rw : 0.0;
    l.r.tr_y = rh ? (l.r.tr_y - G.region.bly) / rh : 0.0;
    l.r.blx = rw ? (l.r.blx - G.region.blx) / rw : 0.0;
    l.r.bly = rh ? (l.r.bly - G.region.bly) / rh : 0.0;
    l.r.trx *= double(G.cols); l.r.tr_y *= double(G.rows);
    l.r.blx *= double(G.cols); l.r.bly *= double(G.rows);
    const bool along_x = l.r.width() > l.r.height();
    const double grad = along_x ? l.sign() * l.r.height() / l.r.width() : l.sign() * l.r.width() / l.r.height();
    const double constant = along_x ? l.ay() - grad * l.ax() : l.ax() - grad * l.ay();
    const double lo = along_x ? l.ax() : l.r.bly, hi = along_x ? l.bx() : l.r.tr_y;
    const int first = cvt_i32_x86(floor(lo - tol)), last = cvt_i32_x86(floor(hi + tol));
    const int lim = along_x ? G.cols : G.rows, olim = along_x ? G.rows : G.cols;
    const int ib = max(first, 0), ie = min(last, lim - 1);
    for (int i = ib; i <= ie; i++) {
        const int j1 = cvt_i32_x86(floor((first == i ? lo : double(i)) * grad + constant - l.sign() * tol));
        const int j2 = cvt_i32_x86(floor((last == i ? hi : double(i + 1)) * grad + constant + l.sign() * tol));
        const int js[3] = {j1, j2, (int)(((long long)j1 + j2) / 2)};
        const int nj = (j1 != j2) ? (abs(j2 - j1) == 2 ? 3 : 2) : 1;
        for (int k = 0; k < nj; k++) {
            const int j = (short)js[k];
            if (j < 0 || j >= olim) continue;
            emit(along_x ? (int64_t)i * G.rows + j : (int64_t)j * G.rows + i);
        }
    }
}

// Pass 1: touched cells per line.
__global__ void rast_count_kernel(FillGrid G, const double* draw, int64_t L, int64_t* line_cnt) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= L) return;
    int64_t n = 0;
    rasterise_line(G, drawing_seg(draw, k), [&](int64_t) { n++; });
    line_cnt[k] = n;
}

// Pass 2: the (cell, line) emissions, line-major, and the number of lines per cell.
__global__ void rast_emit_kernel(FillGrid G, const double* draw, int64_t L, const int64_t* line_off, int32_t* em_cell,
                                 int64_t* cell_cnt) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= L) return;
    int64_t e = line_off[k];
    rasterise_line(G, drawing_seg(draw, k), [&](int64_t c) {
        em_cell[e++] = (int32_t)c;
        atomicAdd((unsigned long long*)&cell_cnt[c], 1ull);
    });
}

// Pass 3: scatter each emission's line index into its cell's list (order fixed by pass 4).
__global__ void rast_place_kernel(const int64_t* line_off, int64_t L, const int32_t* em_cell, int64_t E,
                                  const int64_t* cell_off, int64_t* cursor, int32_t* cell_lines) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    // the emission's line: last k with line_off[k] <= e (binary search over the L+1 offsets)
    int64_t lo = 0, hi = L - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (line_off[mid] <= e) lo = mid;
        else hi = mid - 1;
    }
    const int32_t c = em_cell[e];
    const unsigned long long slot = atomicAdd((unsigned long long*)&cursor[c], 1ull);
    cell_lines[cell_off[c] + (int64_t)slot] = (int32_t)lo;
}

__device__ __forceinline__ Rect cell_region(const FillGrid& G, int x, int y, double border) {
    // PointMap::regionate (pointdata.h:359-367)
    return Rect{G.blx + G.spacing * (double(x) - 0.5 - border), G.bly + G.spacing * (double(y) - 0.5 - border),
                G.blx + G.spacing * (double(x) + 0.5 + border), G.bly + G.spacing * (double(y) + 0.5 + border)};
}

// Pass 4: per cell, sort its lines into drawing order, mark it BLOCKED, and count the crops that
// survive (Line::crop of every copy; a copy that misses the cell box is dropped).
__global__ void rast_crop_count_kernel(FillGrid G, const double* draw, int64_t C, const int64_t* cell_off,
                                       int32_t* cell_lines, int32_t* state, int64_t* piece_cnt) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const int64_t b = cell_off[c], e = cell_off[c + 1];
    int64_t n = 0;
    if (e > b) {
        for (int64_t i = b + 1; i < e; i++) {   // insertion sort: lists are a few lines long
            const int32_t v = cell_lines[i];
            int64_t j = i - 1;
            while (j >= b && cell_lines[j] > v) { cell_lines[j + 1] = cell_lines[j]; j--; }
            cell_lines[j + 1] = v;
        }
        state[c] |= CELL_BLOCKED;
        const Rect box = cell_region(G, (int)(c / G.rows), (int)(c % G.rows), 1e-10);
        for (int64_t i = b; i < e; i++) {
            Seg s = drawing_seg(draw, cell_lines[i]);
            if (clip_seg(s, box)) n++;
        }
    }
    piece_cnt[c] = n;
}

// Pass 5: write the cropped pieces (start.x, start.y, end.x, end.y) at the cell's offset.
__global__ void rast_crop_write_kernel(FillGrid G, const double* draw, int64_t C, const int64_t* cell_off,
                                       const int32_t* cell_lines, const int64_t* piece_off, double* segs) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const int64_t b = cell_off[c], e = cell_off[c + 1];
    if (e == b) return;
    const Rect box = cell_region(G, (int)(c / G.rows), (int)(c % G.rows), 1e-10);
    int64_t o = piece_off[c];
    for (int64_t i = b; i < e; i++) {
        Seg s = drawing_seg(draw, cell_lines[i]);
        if (!clip_seg(s, box)) continue;
        const Vec2 a = s.start(), z = s.end();
        segs[4 * o] = a.x; segs[4 * o + 1] = a.y; segs[4 * o + 2] = z.x; segs[4 * o + 3] = z.y;
        o++;
    }
}

// expand's direction order (pointdata.cpp:459-466): N, S, W, E, NW, NE, SW, SE.
__constant__ int c_fill_dx[8] = {0, 0, -1, 1, -1, 1, -1, 1};
__constant__ int c_fill_dy[8] = {1, -1, 0, 0, 1, 1, -1, -1};

// expand's occluder test (pointdata.cpp:497-506): the centre-to-centre segment against the cropped
// pieces of both cells, tolerance spacing * 1e-10, touching counts.
__device__ bool fill_step_blocked(const FillGrid& G, const int32_t* seg_off, const double* segs, int x1, int y1,
                                  int x2, int y2) {
    const Seg l = make_seg(Vec2{G.blx + G.spacing * 1.0 * double(x1), G.bly + G.spacing * 1.0 * double(y1)},
                           Vec2{G.blx + G.spacing * 1.0 * double(x2), G.bly + G.spacing * 1.0 * double(y2)});
    const double tol = G.spacing * 1e-10;
    const int64_t cs[2] = {(int64_t)x1 * G.rows + y1, (int64_t)x2 * G.rows + y2};
    for (int t = 0; t < 2; t++)
        for (int32_t k = seg_off[cs[t]]; k < seg_off[cs[t] + 1]; k++) {
            const Seg s = make_seg(Vec2{segs[4 * (int64_t)k], segs[4 * (int64_t)k + 1]},
                                   Vec2{segs[4 * (int64_t)k + 2], segs[4 * (int64_t)k + 3]});
            if (rects_touch(l.r, s.r, tol) && segs_cross(l, s, tol)) return true;
        }
    return false;
}

// Claim: every unblocked expand of layer cell p onto a cell unfilled at the start of the layer bids
// its call index p*8+k; blocked calls are remembered for the edge test.
__device__ __forceinline__ uint32_t fill_claim_one(const FillGrid& G, const int32_t* seg_off, const double* segs,
                                                   const int32_t* state, int32_t c, int64_t p, uint32_t* owner) {
    const int x = c / G.rows, y = c % G.rows;
    uint32_t bm = 0;
    for (int k = 0; k < 8; k++) {
        const int x2 = x + c_fill_dx[k], y2 = y + c_fill_dy[k];
        if (x2 < 0 || x2 >= G.cols || y2 < 0 || y2 >= G.rows) continue;
        const int64_t c2 = (int64_t)x2 * G.rows + y2;
        if (state[c2] & CELL_FILLED) continue;
        if (fill_step_blocked(G, seg_off, segs, x, y, x2, y2)) bm |= 1u << k;
        else atomicMin(&owner[c2], (uint32_t)(p * 8 + k));
    }
    return bm;
}

// Resolve: the edge bit of layer cell p and the neighbours it fills (returned as a direction mask).
// owner is read at agent scope: the bids are atomics, served by L2, never by a stale L1 line.
__device__ __forceinline__ uint32_t fill_resolve_one(const FillGrid& G, int32_t* state, int32_t c, int64_t p,
                                                     const uint32_t* owner, uint32_t blocked) {
    const int x = c / G.rows, y = c % G.rows;
    bool edge = (state[c] & CELL_BLOCKED) != 0;
    uint32_t ch = 0;
    for (int k = 0; k < 8; k++) {
        const int x2 = x + c_fill_dx[k], y2 = y + c_fill_dy[k];
        if (x2 < 0 || x2 >= G.cols || y2 < 0 || y2 >= G.rows) continue;
        const int64_t c2 = (int64_t)x2 * G.rows + y2;
        if (state[c2] & CELL_FILLED) continue;
        const uint32_t me = (uint32_t)(p * 8 + k);
        const uint32_t ow = __hip_atomic_load(&owner[c2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((blocked >> k) & 1) {
            if (!(ow < me)) edge = true;   // expand returned 4
        } else if (ow == me) {
            ch |= 1u << k;                 // expand returned 8
        }
    }
    if (edge) atomicOr(&state[c], (int32_t)CELL_EDGE);
    return ch;
}

// Push: the owned neighbours in direction order at consecutive push positions from q; the next layer
// is processed from the back, so push position q lands at index n_next - 1 - q.
__device__ __forceinline__ void fill_push_one(const FillGrid& G, int32_t* state, int32_t c, uint32_t ch, int64_t q,
                                              int64_t n_next, int32_t* next) {
    const int x = c / G.rows, y = c % G.rows;
    for (int k = 0; k < 8; k++) {
        if (!((ch >> k) & 1)) continue;
        const int64_t c2 = (int64_t)(x + c_fill_dx[k]) * G.rows + (y + c_fill_dy[k]);
        state[c2] = G.fill_state | (state[c2] & CELL_BLOCKED);   // Point::set keeps BLOCKED
        next[n_next - 1 - q] = (int32_t)c2;
        q++;
    }
}

__global__ void fill_claim_kernel(FillGrid G, const int32_t* seg_off, const double* segs, const int32_t* state,
                                  const int32_t* layer, int64_t n, uint32_t* owner, uint8_t* blocked) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    blocked[p] = (uint8_t)fill_claim_one(G, seg_off, segs, state, layer[p], p, owner);
}

__global__ void fill_resolve_kernel(FillGrid G, int32_t* state, const int32_t* layer, int64_t n, const uint32_t* owner,
                                    const uint8_t* blocked, uint8_t* children, int64_t* child_cnt) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint32_t ch = fill_resolve_one(G, state, layer[p], p, owner, blocked[p]);
    children[p] = (uint8_t)ch;
    child_cnt[p] = __popc(ch);
}

__global__ void fill_push_kernel(const FillGrid G, int32_t* state, const int32_t* layer, int64_t n,
                                 const uint8_t* children, const int64_t* child_off, int64_t n_next, int32_t* next) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint32_t ch = children[p];
    if (ch) fill_push_one(G, state, layer[p], ch, child_off[p], n_next, next);
}

// Small layers: one workgroup runs level after level with no host round trip (a launch and an 8-byte
// readback per level cost ~47 us; a workgroup barrier a few hundred ns).  It stops when the fill is
// done or a layer outgrows FILL_WG_CAP cells, leaving {n, cur} in io for the host, which continues with
// the grid-wide kernels above.  Same claim / resolve / push bodies, separated by barriers; the per-cell
// masks live in LDS, and each thread owns a contiguous slice of the layer so that its push positions
// follow from one exclusive scan of the slice counts.
constexpr int FILL_WG_THREADS = 1024, FILL_WG_CAP = 16384;
__global__ void __launch_bounds__(FILL_WG_THREADS) fill_levels_wg_kernel(FillGrid G, const int32_t* seg_off,
                                                                         const double* segs, int32_t* state,
                                                                         int32_t* layer0, int32_t* layer1,
                                                                         uint32_t* owner, long long* io) {
    __shared__ uint8_t blk[FILL_WG_CAP], chm[FILL_WG_CAP];
    __shared__ int part[FILL_WG_THREADS];
    const int tid = threadIdx.x;
    int64_t n = io[0];
    int cur = (int)io[1];
    long long levels = 0;
    while (n > 0 && n <= FILL_WG_CAP) {
        const int32_t* layer = cur ? layer1 : layer0;
        int32_t* next = cur ? layer0 : layer1;
        for (int p = tid; p < n; p += FILL_WG_THREADS) blk[p] = (uint8_t)fill_claim_one(G, seg_off, segs, state, layer[p], p, owner);
        __builtin_amdgcn_s_waitcnt(0);   // the bids (atomics) have reached L2 before anyone resolves
        __syncthreads();
        const int per = (int)((n + FILL_WG_THREADS - 1) / FILL_WG_THREADS);
        const int pb = min((int64_t)tid * per, n), pe = min((int64_t)(tid + 1) * per, n);
        int cnt = 0;
        for (int p = pb; p < pe; p++) {
            const uint32_t ch = fill_resolve_one(G, state, layer[p], p, owner, blk[p]);
            chm[p] = (uint8_t)ch;
            cnt += __popc(ch);
        }
        part[tid] = cnt;
        __syncthreads();
        for (int d = 1; d < FILL_WG_THREADS; d <<= 1) {   // inclusive scan of the slice counts
            const int v = tid >= d ? part[tid - d] : 0;
            __syncthreads();
            part[tid] += v;
            __syncthreads();
        }
        const int64_t n_next = part[FILL_WG_THREADS - 1];
        int64_t q = part[tid] - cnt;
        for (int p = pb; p < pe; p++) {
            const uint32_t ch = chm[p];
            if (ch) fill_push_one(G, state, layer[p], ch, q, n_next, next);
            q += __popc(ch);
        }
        __builtin_amdgcn_s_waitcnt(0);   // the pushed cells and states are stored before the next claim
        __syncthreads();
        n = n_next;
        cur ^= 1;
        levels++;
    }
    if (tid == 0) { io[0] = n; io[1] = cur; io[2] = levels; }
}

// ---- exclusive scan of int64 counts (out[0..n) = prefix, out[n] = total) ----
constexpr int SCAN_THREADS = 256, SCAN_PER_THREAD = 8, SCAN_TILE = SCAN_THREADS * SCAN_PER_THREAD;

__global__ void scan_tile_kernel(const int64_t* in, int64_t n, int64_t* out, int64_t* tile_sum) {
    __shared__ int64_t part[SCAN_THREADS];
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_PER_THREAD;
    int64_t v[SCAN_PER_THREAD], s = 0;
    for (int i = 0; i < SCAN_PER_THREAD; i++) {
        v[i] = (base + i < n) ? in[base + i] : 0;
        s += v[i];
    }
    part[threadIdx.x] = s;
    __syncthreads();
    for (int d = 1; d < SCAN_THREADS; d <<= 1) {   // Hillis-Steele inclusive scan of the thread sums
        const int64_t t = (threadIdx.x >= (unsigned)d) ? part[threadIdx.x - d] : 0;
        __syncthreads();
        part[threadIdx.x] += t;
        __syncthreads();
    }
    int64_t run = part[threadIdx.x] - s;
    for (int i = 0; i < SCAN_PER_THREAD; i++) {
        if (base + i < n) out[base + i] = run;
        run += v[i];
    }
    if (threadIdx.x == SCAN_THREADS - 1) tile_sum[blockIdx.x] = part[threadIdx.x];
}

__global__ void scan_add_kernel(int64_t* out, int64_t n, const int64_t* tile_off) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] += tile_off[i / SCAN_TILE];
}

__global__ void scan_total_kernel(int64_t* out, int64_t n, const int64_t* tile_sum) { out[n] = tile_sum[0]; }

} // namespace dmx
