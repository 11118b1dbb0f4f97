// vga_ordered.hip -- the reference's own level order, for the searches whose result depends on it.
//
// VGAVisualGlobal::run (salalib/vgamodules/vgavisualglobal.cpp:96-128) and VGAVisualGlobalDepth::run
// (vgavisualglobaldepth.cpp:44-69) keep each level as a vector, pop it back to front, and let an expanded
// cell extract its merge partner (Point::m_merge) at once.  Every other search of this engine is level-
// synchronous and exact whatever the order inside a level (common.hpp, merge_level_pass); the one exception
// is a link with one end context-filled at an odd PixelRef (not expanded under a radius / in visual step
// depth) and the other end expandable, both new at the same level: the reference counts the unexpanded end if
// it pops it first and extracts it uncounted if it pops the other end first.  The level-synchronous kernels
// flag such a source (merge_order_check, vsd_pending_kernel) and the host re-runs it here.
//
// One workgroup follows one search in the reference's order: the level vector in HBM scratch, cells popped
// back to front, each expansion (Node::extractUnseen -> Bin::extractUnseen, ngraph.cpp:60-65, :308-326)
// walking the node's runs in bin order.  The workgroup shares each expansion: its threads take consecutive
// runs (a node's runs are disjoint), count the unseen cells of their run, and after a workgroup scan push
// them at their run's offset, so the pushes land in the reference's order.  The extent short cut of
// Bin::extractUnseen (a walk stops at a cell whose extent already reaches the run's end) is kept: it skips
// only cells that are already seen, and it keeps the walk at the reference's cost.
#include "common.hpp"

namespace dmx {

constexpr int ORD_NT = 256;

struct OrderedParams {
    int rows;
    int64_t C, N;
    const int64_t* node_run_start;
    const int32_t* node_nruns;
    const Run* pool;
    const int32_t* cell_node;     // [C] node or -1
    const int32_t* node_cell;     // [N]
    const int32_t* merge_cell;    // [C] merge partner cell or -1 (null: no links)
    const uint8_t* node_flags;    // [N] bit 0: context-filled
    // VGA global (seeds == null): one search per listed source node, radius (-1: n)
    const int32_t* src;
    int nsrc;
    int radius;
    int hmax;                     // levels kept per search (radius + 2, or the deepest search vga_do follows)
    int32_t* hist_all;            // [nsrc][hmax] counted cells per level (by search index)
    int32_t* nlev_all;            // [nsrc] levels
    // visual step depth: one search from the level-0 cells (PixelRef order), levels into cell_level
    const int32_t* seeds;
    int nseeds;
    int32_t* cell_level;          // [C]
    // per-workgroup scratch
    uint8_t* misc;                // [C] 0 unseen, 1 in a level vector, 2 done (the reference's ~0)
    int16_t* ext;                 // [C][2] extent along x (H runs) and y (V runs)
    int32_t* vec;                 // [2][N] level vectors (cells)
    int* error;
    int* work_counter;            // searches are taken from it (zeroed by the host)
    DmxCtl* ctl;                  // progress / cancel block (nullptr: none)
};

__device__ __forceinline__ bool cf_odd(const OrderedParams& P, int c) {
    const int x = c / P.rows, y = c % P.rows;
    const int k = P.cell_node[c];
    return k >= 0 && (P.node_flags[k] & 1) && !((x % 2) == 0 && (y % 2) == 0);
}

// workgroup exclusive scan of v (ORD_NT threads); *total receives the sum
__device__ __forceinline__ int ord_scan(int v, int* wsum, int* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int s = v;
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(s, o);
        if (lane >= o) s += t;
    }
    if (lane == 63) wsum[wave] = s;
    __syncthreads();
    int before = 0, all = 0;
    for (int w = 0; w < ORD_NT / 64; w++) {
        if (w < wave) before += wsum[w];
        all += wsum[w];
    }
    __syncthreads();
    *total = all;
    return before + s - v;
}

// Walk run `ru` from its start as Bin::extractUnseen does (ngraph.cpp:311-324): count (push == false) or push
// (at out[pos...], marking misc and the extents) the unseen cells.  The count pass only reads, so both
// passes stop at the same cell.
__device__ __forceinline__ int ord_walk(const OrderedParams& P, Run ru, bool push, int32_t* out, int pos) {
    const int dir = run_dir(ru);
    int dx, dy;
    dir_step(dir, dx, dy);
    int x = ru.x0, y = ru.y0, n = 0;
    const int endc = (dir == 1) ? ru.y1 : ru.x1;
    for (;;) {
        if (((dir == 1) ? y : x) > endc) break;
        const int64_t c = (int64_t)x * P.rows + y;
        if (P.misc[c] == 0) {
            if (push) {
                out[pos + n] = (int32_t)c;
                P.misc[c] = 1;
            }
            n++;
        }
        if (dir <= 1) {   // H / V: the extent short cut (not along diagonals)
            int16_t& e = P.ext[2 * c + dir];
            if (e >= endc) break;
            if (push) e = (int16_t)endc;
        }
        x += dx;
        y += dy;
    }
    return n;
}

// Node::extractUnseen of node k's runs into out[*nout...] (all threads; returns with *nout advanced)
__device__ __forceinline__ void ord_extract(const OrderedParams& P, int64_t k, int32_t* out, int* nout, int* wsum) {
    const int64_t rs = P.node_run_start[k];
    const int nr = P.node_nruns[k];
    for (int r0 = 0; r0 < nr; r0 += ORD_NT) {
        const int r = r0 + (int)threadIdx.x;
        Run ru{0, 0, -1, -1};
        int cnt = 0;
        if (r < nr) {
            ru = P.pool[rs + r];
            cnt = ord_walk(P, ru, false, nullptr, 0);
        }
        int total = 0;
        const int pos = ord_scan(cnt, wsum, &total);
        const int base = *nout;
        if (r < nr && cnt) ord_walk(P, ru, true, out, base + pos);
        __syncthreads();
        if (threadIdx.x == 0) *nout = base + total;
        __syncthreads();
    }
}

__global__ void __launch_bounds__(ORD_NT) vga_ordered_kernel(const OrderedParams* __restrict__ PP) {
    OrderedParams P = const_params(PP);   // this workgroup's scratch: misc [C], ext [C][2], vec [2][N] per workgroup
    P.misc += (size_t)blockIdx.x * P.C;
    P.ext += (size_t)blockIdx.x * 2 * P.C;
    P.vec += (size_t)blockIdx.x * 2 * P.N;
    __shared__ int wsum[ORD_NT / 64];
    __shared__ int sh_n[2];
    __shared__ int sh_cell, sh_act, sh_si;
    const int tid = threadIdx.x;
    const bool vsd = P.seeds != nullptr;
    const int nsearch = vsd ? 1 : P.nsrc;
    int32_t* vec0 = P.vec;
    int32_t* vec1 = P.vec + P.N;
    for (;;) {   // searches from the shared counter, which also carries the cancel flag (ctl_poll)
        if (tid == 0) sh_si = ctl_poll(P.ctl, atomicAdd(P.work_counter, 1));
        __syncthreads();
        const int si = sh_si;
        if (si >= nsearch) break;
        for (int64_t c = tid; c < P.C; c += ORD_NT) {
            P.misc[c] = 0;
            P.ext[2 * c] = (int16_t)(c / P.rows);
            P.ext[2 * c + 1] = (int16_t)(c % P.rows);
        }
        __syncthreads();
        int64_t src = -1;
        if (vsd) {
            for (int i = tid; i < P.nseeds; i += ORD_NT) vec0[i] = P.seeds[i];
            if (tid == 0) sh_n[0] = P.nseeds;
        } else {
            src = P.src[si];
            if (tid == 0) { vec0[0] = P.node_cell[src]; sh_n[0] = 1; }
        }
        __syncthreads();
        int32_t* cur = vec0;
        int32_t* nxt = vec1;
        int level = 0;
        while (sh_n[0] > 0) {
            const int ncur = sh_n[0];
            if (tid == 0) sh_n[1] = 0;
            int counted = 0;   // (thread 0)
            __syncthreads();
            for (int i = ncur - 1; i >= 0; i--) {   // back to front (rbegin .. rend)
                if (tid == 0) {
                    const int c = cur[i];
                    int act = 0;   // 0 skip, 1 counted and expanded, 2 counted only
                    if (P.misc[c] != 2) {
                        const bool expand = vsd ? (level == 0 || !cf_odd(P, c))
                                                : (P.radius == -1 || (level < P.radius && !cf_odd(P, c)));
                        act = expand ? 1 : 2;
                        counted++;
                        if (vsd) P.cell_level[c] = level;
                        if (!expand) P.misc[c] = 2;
                    }
                    sh_cell = c;
                    sh_act = act;
                }
                __syncthreads();
                const int c = sh_cell, act = sh_act;
                if (act == 1) {
                    ord_extract(P, P.cell_node[c], nxt, &sh_n[1], wsum);
                    if (tid == 0) P.misc[c] = 2;
                    __syncthreads();
                    const int m = P.merge_cell ? P.merge_cell[c] : -1;
                    if (m >= 0 && P.misc[m] != 2) {   // getMergePixel (vgavisualglobal.cpp:113-122)
                        if (vsd && tid == 0) P.cell_level[m] = level;
                        ord_extract(P, P.cell_node[m], nxt, &sh_n[1], wsum);
                        if (tid == 0) P.misc[m] = 2;
                    }
                }
                __syncthreads();
            }
            if (!vsd && tid == 0) {
                if (level < P.hmax) P.hist_all[(int64_t)si * P.hmax + level] = counted;
                else atomicOr(P.error, KERR_LEVELS);
            }
            level++;
            if (tid == 0) sh_n[0] = sh_n[1];
            int32_t* t = cur; cur = nxt; nxt = t;
            __syncthreads();
        }
        if (!vsd && tid == 0) P.nlev_all[si] = min(level, P.hmax);
        __syncthreads();
    }
}

} // namespace dmx
