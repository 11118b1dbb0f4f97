// vga.hip -- K3/K4: VGA global visibility (all-sources level BFS + integration measures) on gfx950.
//
// Replaces VGAVisualGlobal::run / extractUnseen (salalib/vgamodules/vgavisualglobal.cpp:23-240) and
// the measure formulas of genlib/pafmath.h:59-80.
//
// The reference walks every run cell by cell per source with misc/extent matrices that are reset
// over the whole grid for every source.  Its result only depends on set semantics: the cells
// discovered at level L+1 are (union of the run cells of every expanded level-L node) minus the
// cells already seen; a cell is counted once, at the level it is discovered, iff it is FILLED
// (non-filled cells inside diagonal spans are pushed but never counted or expanded).  So here:
//   * one workgroup (4 waves) owns one source at a time (persistent grid, dynamic counter);
//   * the "seen" set is an LDS bitmap tiled in 8x8-cell 64-bit words, pre-seeded with every
//     non-filled cell, so a whole horizontal or vertical run is applied with ~len/8 LDS atomic ORs
//     and every newly set bit is a filled, countable cell;
//   * frontiers are node-index lists in HBM (per workgroup), level counts in LDS;
//   * early exit: once every filled cell that appears in any run (|U_f|, precomputed) is seen,
//     no further expansion can discover anything and the BFS stops;
//   * the 7 measures are computed in FP64 by lane 0 from the level histogram.
#include "common.hpp"

namespace dmx {

struct VgaParams {
    int cols, rows, tw, th;     // tiles per row / column (8x8 cells per 64-bit word)
    const unsigned long long* seed_tiles;   // [tw*th] 1 = non-filled cell (or padding)
    const unsigned long long* uf_tiles;     // [tw*th] 1 = filled cell appearing in some run
    int64_t uf_count;           // popcount(uf_tiles)
    const int32_t* node_cell;   // [N]
    const int32_t* cell_node;   // [C] x-major -> node or -1
    const uint8_t* node_flags;  // [N] bit0 CONTEXTFILLED
    const int64_t* node_run_start;
    const int32_t* node_nruns;
    const Run* pool;
    int64_t src_begin, src_end;
    int radius;                 // -1 = n
    int gates_only;
    int* work_counter;
    int32_t* frontier;          // per workgroup: 2 * nnodes
    int64_t nnodes;
    int maxlev;
    float* out;                 // [N][7] (indexed by node)
    int64_t* levels_out;        // optional [N][3]: total nodes, total depth, levels
    int* error;
    unsigned long long* stats;  // [0] runs expanded, [1] LDS tile words touched, [2] cells reached
};

__device__ __forceinline__ double plog2(double a) { return log(a) * 1.4426950408889634073599246810019; } // pafmath.h:61
__device__ __forceinline__ double dvalue(double k) { // pafmath.h:72
    return 2.0 * (k * (plog2((k + 2.0) / 3.0) - 1.0) + 1.0) / ((k - 1.0) * (k - 2.0));
}
__device__ __forceinline__ double pvalue(double k) { return 2.0 * (k - plog2(k) - 1.0) / ((k - 1.0) * (k - 2.0)); }
__device__ __forceinline__ double teklinteg(double nc, double td) { return log(0.5 * (nc - 2.0)) / log(double(td - nc + 1)); }

constexpr int VGA_THREADS = 256;

struct VgaShared {
    int next_item;
    int stop;
    int nnext;
    int pad;
    unsigned long long seen_filled;
};

// Apply one tile word: returns the newly-set bits, appends their nodes to the next frontier.
__device__ __forceinline__ void apply_word(unsigned long long* tiles, int tw, int tx, int ty, unsigned long long mask,
                                           const VgaParams& P, int rows, VgaShared* S, int32_t* next, int cap,
                                           int& local_new) {
    const int w = ty * tw + tx;
    unsigned long long old = atomicOr(&tiles[w], mask);
    unsigned long long nw = mask & ~old;
    if (nw) {
        const int c = __popcll(nw);
        local_new += c;
        int pos = atomicAdd(&S->nnext, c);
        while (nw) {
            const int b = __ffsll((long long)nw) - 1;
            nw &= nw - 1;
            const int x = tx * 8 + (b & 7), y = ty * 8 + (b >> 3);
            if (pos < cap) next[pos] = P.cell_node[x * rows + y];
            pos++;
        }
    }
}

__global__ void __launch_bounds__(VGA_THREADS) vga_global_kernel(VgaParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int ntiles = P.tw * P.th;
    unsigned long long* tiles = (unsigned long long*)smem;
    int* hist = (int*)(tiles + ntiles);
    VgaShared* S = (VgaShared*)(hist + P.maxlev + 4);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int cap = (int)P.nnodes;
    int32_t* fa = P.frontier + (size_t)blockIdx.x * 2 * P.nnodes;
    int32_t* fb = fa + P.nnodes;
    __shared__ int s_src;

    for (;;) {
        if (tid == 0) s_src = atomicAdd(P.work_counter, 1);
        __syncthreads();
        const int64_t src = P.src_begin + s_src;
        __syncthreads();
        if (src >= P.src_end) break;
        float* o = P.out + src * 7;
        const int scell = P.node_cell[src];
        const int sx = scell / P.rows, sy = scell % P.rows;
        const bool sctx = P.node_flags[src] & 1;
        // VGAVisualGlobal::run: context-filled odd cells and gates_only are skipped (:72-75)
        if ((sctx && !((sx % 2) == 0 && (sy % 2) == 0)) || P.gates_only) {
            if (tid < 7) o[tid] = -1.0f;
            if (P.levels_out && tid < 3) P.levels_out[src * 3 + tid] = 0;
            continue;
        }
        for (int i = tid; i < ntiles; i += VGA_THREADS) tiles[i] = P.seed_tiles[i];
        for (int i = tid; i < P.maxlev + 4; i += VGA_THREADS) hist[i] = 0;
        if (tid == 0) { S->stop = 0; S->nnext = 0; S->next_item = 0; S->seen_filled = 1; }
        __syncthreads();
        const int stile = (sy >> 3) * P.tw + (sx >> 3);
        const unsigned long long sbit = 1ull << ((sy & 7) * 8 + (sx & 7));
        if (tid == 0) {
            tiles[stile] |= sbit;
            fa[0] = (int32_t)src;
            hist[0] = 1;
        }
        const bool s_in_uf = (P.uf_tiles[stile] & sbit) != 0;
        const unsigned long long target = (unsigned long long)P.uf_count + (s_in_uf ? 0 : 1);
        __syncthreads();
        int nfront = 1, level = 0, nlev = 1;
        bool overflow = false;
        while (nfront > 0) {
            const bool expand_level = (P.radius == -1) || (level < P.radius);
            if (!expand_level || *(volatile int*)&S->stop) break;
            // ---- expand every node of this level (work items = nodes, one wave at a time)
            for (;;) {
                int item = 0;
                if (lane == 0) item = atomicAdd(&S->next_item, 1);
                item = __shfl(item, 0);
                if (item >= nfront || *(volatile int*)&S->stop) break;
                const int node = fa[item];
                if (P.radius != -1) {
                    // radius-limited: context-filled odd cells are not expanded (:104-107)
                    const int c = P.node_cell[node];
                    const int nx = c / P.rows, ny = c % P.rows;
                    if ((P.node_flags[node] & 1) && !((nx % 2) == 0 && (ny % 2) == 0)) continue;
                }
                const int64_t rs = P.node_run_start[node];
                const int nr = P.node_nruns[node];
                int local_new = 0;
                if (lane == 0) atomicAdd(&P.stats[0], (unsigned long long)nr);
                for (int r = lane; r < nr; r += 64) {
                    const Run ru = P.pool[rs + r];
                    if (ru.y0 == ru.y1 && ru.x0 != ru.x1) { // horizontal
                        const int y = ru.y0, ty = y >> 3, sh = (y & 7) * 8;
                        for (int tx = ru.x0 >> 3; tx <= (ru.x1 >> 3); tx++) {
                            const int lo = max((int)ru.x0, tx * 8) & 7, hi = min((int)ru.x1, tx * 8 + 7) & 7;
                            const unsigned long long m = (unsigned long long)((0xFFu >> (7 - hi)) & (0xFFu << lo) & 0xFFu) << sh;
                            apply_word(tiles, P.tw, tx, ty, m, P, P.rows, S, fb, cap, local_new);
                        }
                    } else if (ru.x0 == ru.x1 && ru.y0 != ru.y1) { // vertical
                        const int x = ru.x0, tx = x >> 3;
                        const unsigned long long col = 0x0101010101010101ull << (x & 7);
                        for (int ty = ru.y0 >> 3; ty <= (ru.y1 >> 3); ty++) {
                            const int lo = max((int)ru.y0, ty * 8) & 7, hi = min((int)ru.y1, ty * 8 + 7) & 7;
                            const unsigned long long rows = (~0ull >> (8 * (7 - hi))) & (~0ull << (8 * lo));
                            apply_word(tiles, P.tw, tx, ty, col & rows, P, P.rows, S, fb, cap, local_new);
                        }
                    } else { // diagonal span (gaps included) or single cell
                        const int dy = (ru.y1 > ru.y0) ? 1 : ((ru.y1 < ru.y0) ? -1 : 0);
                        int y = ru.y0;
                        for (int x = ru.x0; x <= ru.x1; x++, y += dy) {
                            apply_word(tiles, P.tw, x >> 3, y >> 3, 1ull << ((y & 7) * 8 + (x & 7)), P, P.rows, S, fb,
                                       cap, local_new);
                        }
                    }
                }
                // wave total of new cells -> early exit test
                for (int off = 32; off >= 1; off >>= 1) local_new += __shfl_xor(local_new, off);
                if (lane == 0 && local_new) {
                    unsigned long long tot = atomicAdd(&S->seen_filled, (unsigned long long)local_new) + local_new;
                    if (tot >= target) S->stop = 1;
                }
            }
            __syncthreads();
            const int nn = S->nnext;
            if (nn > cap) overflow = true;
            __syncthreads();
            if (tid == 0) {
                S->nnext = 0;
                S->next_item = 0;
                if (level + 1 < P.maxlev) hist[level + 1] = nn;
            }
            if (level + 1 >= P.maxlev) overflow = true;
            __syncthreads();
            if (overflow) break;
            int32_t* t = fa; fa = fb; fb = t;
            nfront = nn;
            level++;
            if (nn > 0) nlev = level + 1;
        }
        if (overflow) {
            if (tid == 0) atomicOr(P.error, KERR_FRONTIER);
            continue;
        }
        // ---- measures (vgavisualglobal.cpp:131-193), lane 0 in FP64
        if (tid == 0) {
            long long total_nodes = 0, total_depth = 0;
            for (int l = 0; l < nlev; l++) { total_nodes += hist[l]; total_depth += (long long)l * hist[l]; }
            float r[7];
            for (int i = 0; i < 7; i++) r[i] = -1.0f;
            r[5] = (float)total_nodes;
            if (total_nodes > 1) {
                const double mean_depth = (double)total_depth / (double)(total_nodes - 1);
                r[4] = (float)mean_depth;
                if (total_nodes > 2 && mean_depth > 1.0) {
                    const double ra = 2.0 * (mean_depth - 1.0) / (double)(total_nodes - 2);
                    const double rra_d = ra / dvalue((double)total_nodes);
                    const double rra_p = ra / pvalue((double)total_nodes);
                    const double integ_tk = teklinteg((double)total_nodes, (double)total_depth);
                    r[1] = (float)(1.0 / rra_d);
                    r[2] = (float)(1.0 / rra_p);
                    r[3] = (total_depth - total_nodes + 1 > 1) ? (float)integ_tk : -1.0f;
                }
                double entropy = 0.0, rel_entropy = 0.0, factorial = 1.0;
                for (int k = 1; k < nlev; k++) {
                    if (hist[k] > 0) {
                        const double prob = (double)hist[k] / (double)(total_nodes - 1);
                        entropy -= prob * plog2(prob);
                        factorial *= (double)(k + 1);
                        const double q = (pow(mean_depth, (double)k) / factorial) * exp(-mean_depth);
                        rel_entropy += (double)(float)prob * plog2(prob / q);
                    }
                }
                r[0] = (float)entropy;
                r[6] = (float)rel_entropy;
            }
            for (int i = 0; i < 7; i++) o[i] = r[i];
            atomicAdd(&P.stats[2], (unsigned long long)total_nodes);
            if (P.levels_out) {
                P.levels_out[src * 3 + 0] = total_nodes;
                P.levels_out[src * 3 + 1] = total_depth;
                P.levels_out[src * 3 + 2] = nlev;
            }
        }
        __syncthreads();
    }
}

// U_f: filled cells that appear in at least one run of any node (early-exit target for the BFS).
__global__ void mark_runs_kernel(int tw, const int64_t* node_run_start, const int32_t* node_nruns, const Run* pool,
                                 int64_t n, unsigned long long* tiles) {
    int64_t k = (int64_t)blockIdx.x;
    if (k >= n) return;
    const int64_t rs = node_run_start[k];
    const int nr = node_nruns[k];
    for (int r = threadIdx.x; r < nr; r += blockDim.x) {
        const Run ru = pool[rs + r];
        const int dx = (ru.x1 > ru.x0) ? 1 : 0;
        const int dy = (ru.x0 == ru.x1) ? ((ru.y1 > ru.y0) ? 1 : 0) : ((ru.y1 > ru.y0) ? 1 : ((ru.y1 < ru.y0) ? -1 : 0));
        int x = ru.x0, y = ru.y0;
        for (;;) {
            atomicOr(&tiles[(y >> 3) * tw + (x >> 3)], 1ull << ((y & 7) * 8 + (x & 7)));
            if (x == ru.x1 && y == ru.y1) break;
            x += dx;
            y += dy;
        }
    }
}

} // namespace dmx
