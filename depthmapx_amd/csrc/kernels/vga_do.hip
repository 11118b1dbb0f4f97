// vga_do.hip -- K3 v2: direction-optimising VGA global BFS (+ K4 measures) on gfx950.
//
// Same result as vga.hip's top-down kernel (VGAVisualGlobal::run, vgavisualglobal.cpp:23-216),
// much less work: after level 1 the frontier of an open plan holds a third of the grid and nearly
// every unvisited cell sees one of its members, so instead of expanding every frontier node
// ("top-down", reads all their runs) each unvisited cell scans ITS OWN runs until one touches the
// frontier ("bottom-up", usually a handful of run reads).  Bottom-up is only valid when the
// visibility relation is symmetric (u in cells(v) <=> v in cells(u) over filled cells), which the
// host establishes per graph (symmetry_hash_kernel); otherwise the kernel stays top-down.
//
// Per workgroup (one source at a time, persistent grid): three LDS bitmaps tiled 8x8 cells per
// 64-bit word -- V (seen, pre-seeded with cells that can never be discovered), F (expandable
// frontier) and X (next level).  Per level the direction is chosen with Beamer's test on cell
// counts (n_frontier * alpha > n_unvisited).  Bottom-up cells scan their runs longest-first (the
// scan pool) on their own lane for at most `kshort` runs; the rest go to a hard list scanned 64
// runs at a time per wave.
#include "common.hpp"

namespace dmx {

struct VgaDoParams {
    int cols, rows, tw, th;
    const unsigned long long* seed_tiles;    // non-filled cells, padding, filled cells in no run
    const unsigned long long* uf_tiles;      // filled cells that appear in some run
    const unsigned long long* nonexp_tiles;  // contextfilled odd cells (used when radius != -1)
    const int32_t* node_cell;
    const int32_t* cell_node;
    const uint8_t* node_flags;
    const int64_t* node_run_start;
    const int32_t* node_nruns;
    const Run* pool;
    const int64_t* cell_scan_start;  // [C] start of the cell's runs in scan_pool (longest first)
    const int32_t* cell_nruns;       // [C] (0 for non-filled cells)
    const Run* scan_pool;
    int64_t src_begin, src_end;
    int radius, gates_only;
    int64_t uf_count;       // |U_f|
    int symmetric;          // bottom-up allowed
    // exact in-set corrections for the few nodes whose visibility is not symmetric
    const int32_t* spec_index;    // [N] node -> special index or -1
    const int32_t* extra_off;     // [nspec+1] in-neighbours outside cells(v)
    const int32_t* extra;         // node indices
    const int32_t* missing_off;   // [nspec+1] members of cells(v) that are not in-neighbours
    const int32_t* missing;       // node indices
    int alpha, kshort;
    int* work_counter;
    int32_t* scratch;       // per workgroup: 2 * nnodes ints (cell list + hard list)
    int64_t nnodes;
    int maxlev;
    float* out;
    int64_t* levels_out;
    int* error;
    unsigned long long* stats;  // [0] runs read, [2] cells reached, [3] bottom-up levels, [4] top-down levels,
                                // [5] bottom-up cells that scanned every run without a hit, [6] their runs
    unsigned long long* gbm;    // GBM variant: per workgroup 3*tw*th words (V, F, X) in HBM
    const int2* mpairs;         // [nmp] merge links (cell a, cell b), x-major (nullptr: none)
    int nmp;
    const int2* mamb;           // [nmamb] links with a context-filled odd end (merge_order_check)
    int nmamb = 0;
    int32_t* mseen = nullptr;   // per workgroup [nmamb]
    uint8_t* oflag = nullptr;   // [N] sources whose result depends on the reference's pop order
};

constexpr int DO_THREADS = 256;

__device__ __forceinline__ double do_plog2(double a) { return log(a) * 1.4426950408889634073599246810019; }

// VGAVisualGlobal measures (vgavisualglobal.cpp:131-193) from the level histogram.
__device__ __noinline__ void vga_measures(const int* hist, int nlev, float* o, long long& tn, long long& td) {
    long long total_nodes = 0, total_depth = 0;
    for (int l = 0; l < nlev; l++) { total_nodes += hist[l]; total_depth += (long long)l * hist[l]; }
    float r[7];
    for (int i = 0; i < 7; i++) r[i] = -1.0f;
    r[5] = (float)total_nodes;
    if (total_nodes > 1) {
        const double mean_depth = (double)total_depth / (double)(total_nodes - 1);
        r[4] = (float)mean_depth;
        if (total_nodes > 2 && mean_depth > 1.0) {
            const double k = (double)total_nodes;
            const double ra = 2.0 * (mean_depth - 1.0) / (double)(total_nodes - 2);
            const double dv = 2.0 * (k * (do_plog2((k + 2.0) / 3.0) - 1.0) + 1.0) / ((k - 1.0) * (k - 2.0));
            const double pv = 2.0 * (k - do_plog2(k) - 1.0) / ((k - 1.0) * (k - 2.0));
            const double integ_tk = log(0.5 * (k - 2.0)) / log((double)total_depth - k + 1);
            r[1] = (float)(1.0 / (ra / dv));
            r[2] = (float)(1.0 / (ra / pv));
            r[3] = (total_depth - total_nodes + 1 > 1) ? (float)integ_tk : -1.0f;
        }
        double entropy = 0.0, rel_entropy = 0.0, factorial = 1.0;
        for (int l = 1; l < nlev; l++) {
            if (hist[l] > 0) {
                const double prob = (double)hist[l] / (double)(total_nodes - 1);
                entropy -= prob * do_plog2(prob);
                factorial *= (double)(l + 1);
                const double q = (pow(mean_depth, (double)l) / factorial) * exp(-mean_depth);
                rel_entropy += (double)(float)prob * do_plog2(prob / q);
            }
        }
        r[0] = (float)entropy;
        r[6] = (float)rel_entropy;
    }
    for (int i = 0; i < 7; i++) o[i] = r[i];
    tn = total_nodes;
    td = total_depth;
}

// Does run `ru` touch any bit of the tiled bitmap `bm`?
__device__ __forceinline__ bool run_hits(const unsigned long long* bm, int tw, Run ru) {
    if (ru.y0 == ru.y1 && ru.x0 != ru.x1) {
        const int y = ru.y0, rowoff = (y >> 3) * tw, sh = (y & 7) * 8;
        for (int tx = ru.x0 >> 3; tx <= (ru.x1 >> 3); tx++) {
            const int lo = max((int)ru.x0, tx * 8) & 7, hi = min((int)ru.x1, tx * 8 + 7) & 7;
            const unsigned long long m = (unsigned long long)((0xFFu >> (7 - hi)) & (0xFFu << lo) & 0xFFu) << sh;
            if (bm[rowoff + tx] & m) return true;
        }
        return false;
    } else if (ru.x0 == ru.x1 && ru.y0 != ru.y1) {
        const int x = ru.x0, tx = x >> 3;
        const unsigned long long col = 0x0101010101010101ull << (x & 7);
        for (int ty = ru.y0 >> 3; ty <= (ru.y1 >> 3); ty++) {
            const int lo = max((int)ru.y0, ty * 8) & 7, hi = min((int)ru.y1, ty * 8 + 7) & 7;
            const unsigned long long rws = (~0ull >> (8 * (7 - hi))) & (~0ull << (8 * lo));
            if (bm[ty * tw + tx] & col & rws) return true;
        }
        return false;
    } else {
        const int dy = (ru.y1 > ru.y0) ? 1 : ((ru.y1 < ru.y0) ? -1 : 0);
        int y = ru.y0;
        for (int x = ru.x0; x <= ru.x1; x++, y += dy)
            if (bm[(y >> 3) * tw + (x >> 3)] & (1ull << ((y & 7) * 8 + (x & 7)))) return true;
        return false;
    }
}

// Top-down application of one run: set bits in V, record new bits in X; returns #new cells.
__device__ __forceinline__ int run_push(unsigned long long* V, unsigned long long* X, int tw, Run ru) {
    int nnew = 0;
    auto apply = [&](int w, unsigned long long m) {
        const unsigned long long old = atomicOr(&V[w], m);
        const unsigned long long nw = m & ~old;
        if (nw) { atomicOr(&X[w], nw); nnew += __popcll(nw); }
    };
    if (ru.y0 == ru.y1 && ru.x0 != ru.x1) {
        const int y = ru.y0, rowoff = (y >> 3) * tw, sh = (y & 7) * 8;
        for (int tx = ru.x0 >> 3; tx <= (ru.x1 >> 3); tx++) {
            const int lo = max((int)ru.x0, tx * 8) & 7, hi = min((int)ru.x1, tx * 8 + 7) & 7;
            apply(rowoff + tx, (unsigned long long)((0xFFu >> (7 - hi)) & (0xFFu << lo) & 0xFFu) << sh);
        }
    } else if (ru.x0 == ru.x1 && ru.y0 != ru.y1) {
        const int x = ru.x0, tx = x >> 3;
        const unsigned long long col = 0x0101010101010101ull << (x & 7);
        for (int ty = ru.y0 >> 3; ty <= (ru.y1 >> 3); ty++) {
            const int lo = max((int)ru.y0, ty * 8) & 7, hi = min((int)ru.y1, ty * 8 + 7) & 7;
            apply(ty * tw + tx, col & (~0ull >> (8 * (7 - hi))) & (~0ull << (8 * lo)));
        }
    } else {
        const int dy = (ru.y1 > ru.y0) ? 1 : ((ru.y1 < ru.y0) ? -1 : 0);
        int y = ru.y0;
        for (int x = ru.x0; x <= ru.x1; x++, y += dy) apply((y >> 3) * tw + (x >> 3), 1ull << ((y & 7) * 8 + (x & 7)));
    }
    return nnew;
}

struct DoShared {
    int list_n, hard_n, item, mpart;
    unsigned long long cnt, mass;   // next-level count and its expandable part
    unsigned long long tdnew;       // cells discovered so far in a top-down level
    unsigned long long mcorr, mdisc;   // merge pass (vga_tile.hip, merge_level_pass)
};

// GBM = false: V/F/X bitmaps in LDS (grids up to ~1.7e5 cells); true: in HBM (per-workgroup slice).
template <bool GBM>
__global__ void __launch_bounds__(DO_THREADS) vga_do_kernel(VgaDoParams P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nt = P.tw * P.th;
    unsigned long long* V = GBM ? P.gbm + (size_t)blockIdx.x * 3 * nt : (unsigned long long*)smem;
    unsigned long long* F = V + nt;
    unsigned long long* X = F + nt;
    int* hist = GBM ? (int*)smem : (int*)(X + nt);
    DoShared* S = (DoShared*)(hist + P.maxlev + 4);
    __shared__ int s_src;
    const int tid = threadIdx.x, lane = tid & 63;
    int32_t* list = P.scratch + (size_t)blockIdx.x * 2 * P.nnodes;
    int32_t* hard = list + P.nnodes;
    const int rows = P.rows, tw = P.tw;
    unsigned long long runs_read = 0, fail_cells = 0, fail_runs = 0;

    for (;;) {
        if (tid == 0) s_src = atomicAdd(P.work_counter, 1);
        __syncthreads();
        const int64_t src = P.src_begin + s_src;
        __syncthreads();
        if (src >= P.src_end) break;
        float* o = P.out + src * 7;
        const int scell = P.node_cell[src];
        const int sx = scell / rows, sy = scell % rows;
        if (((P.node_flags[src] & 1) && !((sx % 2) == 0 && (sy % 2) == 0)) || P.gates_only) {
            if (tid < 7) o[tid] = -1.0f;
            if (P.levels_out && tid < 3) P.levels_out[src * 3 + tid] = 0;
            continue;
        }
        const int stile = (sy >> 3) * tw + (sx >> 3);
        const unsigned long long sbit = 1ull << ((sy & 7) * 8 + (sx & 7));
        for (int i = tid; i < nt; i += DO_THREADS) {
            unsigned long long v = P.seed_tiles[i];
            if (i == stile) v |= sbit;
            V[i] = v;
            F[i] = (i == stile) ? sbit : 0ull;
            X[i] = 0ull;
        }
        for (int i = tid; i < P.maxlev + 4; i += DO_THREADS) hist[i] = 0;
        if (tid == 0) {
            hist[0] = 1; S->cnt = 0; S->mass = 0; S->list_n = 0; S->hard_n = 0; S->item = 0; S->tdnew = 0;
            S->mpart = -1; S->mcorr = 0; S->mdisc = 0;
        }
        const bool s_in_uf = (P.uf_tiles[stile] & sbit) != 0;
        long long target = P.uf_count - (s_in_uf ? 1 : 0); // cells still to discover
        long long m_f = 1;
        if (P.nmp) {
            // the source's merge partner is extracted at level 0, uncounted (vgavisualglobal.cpp:113-122)
            __syncthreads();
            for (int i = tid; i < P.nmp; i += DO_THREADS) {
                const int2 pr = P.mpairs[i];
                if (pr.x == scell) S->mpart = pr.y;
                else if (pr.y == scell) S->mpart = pr.x;
            }
            __syncthreads();
            const int pc = S->mpart;
            if (pc >= 0) {
                const int px = pc / rows, py = pc % rows;
                const int pt = (py >> 3) * tw + (px >> 3);
                const unsigned long long pb = 1ull << ((py & 7) * 8 + (px & 7));
                if (tid == 0) { V[pt] |= pb; F[pt] |= pb; }
                if (P.uf_tiles[pt] & pb) target--;
                m_f = 2;
            }
        }
        // Beamer's direction test on cell counts: frontier size vs cells still unvisited
        long long m_u = target;
        long long discovered = 0;
        int level = 0, nlev = 1;
        bool overflow = false;
        __syncthreads();
        for (;;) {
            if (P.radius != -1 && level >= P.radius) break;
            if (discovered >= target) break;
            const bool bottom_up = P.symmetric && level > 0 && (m_f * (long long)P.alpha > m_u);
            if (bottom_up) {
                // ---- list the unvisited cells (every one of them is a filled, discoverable cell)
                for (int i = tid; i < nt; i += DO_THREADS) {
                    unsigned long long u = ~V[i];
                    if (u) {
                        int pos = atomicAdd(&S->list_n, __popcll(u));
                        const int tx = i % tw, ty = i / tw;
                        while (u) {
                            const int b = __ffsll((long long)u) - 1;
                            u &= u - 1;
                            list[pos++] = (tx * 8 + (b & 7)) * rows + ty * 8 + (b >> 3);
                        }
                    }
                }
                __syncthreads();
                const int nl = S->list_n;
                // ---- phase 1: one lane per cell, at most kshort runs
                for (int i = tid; i < nl; i += DO_THREADS) {
                    const int c = list[i];
                    if (P.spec_index && P.spec_index[P.cell_node[c]] >= 0) { // exact path (phase 2)
                        hard[atomicAdd(&S->hard_n, 1)] = -1 - c;
                        continue;
                    }
                    const int64_t rs = P.cell_scan_start[c];
                    const int nr = P.cell_nruns[c];
                    const int lim = min(nr, P.kshort);
                    bool hit = false;
                    int r = 0;
                    for (; r < lim && !hit; r++) hit = run_hits(F, tw, P.scan_pool[rs + r]);
                    runs_read += r;
                    if (hit) {
                        const int x = c / rows, y = c % rows;
                        atomicOr(&X[(y >> 3) * tw + (x >> 3)], 1ull << ((y & 7) * 8 + (x & 7)));
                    } else if (nr > lim) {
                        hard[atomicAdd(&S->hard_n, 1)] = c;
                    } else {
                        fail_cells++;
                        fail_runs += nr;
                    }
                }
                __syncthreads();
                // ---- phase 2: hard cells, a wave scans 64 runs at a time
                const int nh = S->hard_n;
                for (;;) {
                    int it = 0;
                    if (lane == 0) it = atomicAdd(&S->item, 1);
                    it = __shfl(it, 0);
                    if (it >= nh) break;
                    int c = hard[it];
                    const bool special = c < 0;
                    if (special) c = -1 - c;
                    const int node = P.cell_node[c];
                    const int64_t rs = P.node_run_start[node];
                    const int nr = P.node_nruns[node];
                    bool found = false;
                    if (special) {
                        // hit iff some frontier cell u is an in-neighbour: u in Extra(v), or
                        // u in cells(v) and u not in Missing(v)
                        const int si = P.spec_index[node];
                        const int e0 = P.extra_off[si], e1 = P.extra_off[si + 1];
                        const int m0 = P.missing_off[si], m1 = P.missing_off[si + 1];
                        bool h = false;
                        for (int j = e0 + lane; j < e1; j += 64) {
                            const int uc = P.node_cell[P.extra[j]];
                            const int ux = uc / rows, uy = uc % rows;
                            if (F[(uy >> 3) * tw + (ux >> 3)] & (1ull << ((uy & 7) * 8 + (ux & 7)))) h = true;
                        }
                        for (int r = lane; r < nr && !h; r += 64) {
                            const Run ru = P.pool[rs + r];
                            const int dx = (ru.x1 > ru.x0) ? 1 : 0;
                            const int dy = (ru.y0 == ru.y1) ? 0 : ((ru.x0 == ru.x1) ? 1 : ((ru.y1 > ru.y0) ? 1 : -1));
                            int x = ru.x0, y = ru.y0;
                            for (;;) {
                                if (F[(y >> 3) * tw + (x >> 3)] & (1ull << ((y & 7) * 8 + (x & 7)))) {
                                    const int un = P.cell_node[x * rows + y];
                                    bool miss = false;
                                    for (int j = m0; j < m1; j++) miss |= (P.missing[j] == un);
                                    if (!miss) { h = true; break; }
                                }
                                if (x == ru.x1 && y == ru.y1) break;
                                x += dx;
                                y += dy;
                            }
                        }
                        found = __ballot(h) != 0ull;
                        if (lane == 0) runs_read += (unsigned long long)nr;
                    }
                    const int64_t srs = P.cell_scan_start[c];
                    for (int base = P.kshort; base < nr && !found && !special; base += 64) {
                        const int r = base + lane;
                        const bool h = (r < nr) && run_hits(F, tw, P.scan_pool[srs + r]);
                        found = __ballot(h) != 0ull;
                        if (lane == 0) runs_read += (unsigned long long)min(64, nr - base);
                    }
                    if (found && lane == 0) {
                        const int x = c / rows, y = c % rows;
                        atomicOr(&X[(y >> 3) * tw + (x >> 3)], 1ull << ((y & 7) * 8 + (x & 7)));
                    }
                    if (!found && lane == 0) { fail_cells++; fail_runs += nr; }
                }
                __syncthreads();
                for (int i = tid; i < nt; i += DO_THREADS) V[i] |= X[i];
                if (tid == 0) { S->list_n = 0; S->hard_n = 0; S->item = 0; }
            } else {
                // ---- top-down: list the frontier, expand node runs into V / X
                for (int i = tid; i < nt; i += DO_THREADS) {
                    unsigned long long u = F[i];
                    if (u) {
                        int pos = atomicAdd(&S->list_n, __popcll(u));
                        const int tx = i % tw, ty = i / tw;
                        while (u) {
                            const int b = __ffsll((long long)u) - 1;
                            u &= u - 1;
                            list[pos++] = (tx * 8 + (b & 7)) * rows + ty * 8 + (b >> 3);
                        }
                    }
                }
                __syncthreads();
                const int nl = S->list_n;
                for (;;) {
                    int it = 0;
                    if (lane == 0) it = atomicAdd(&S->item, 1);
                    it = __shfl(it, 0);
                    // everything discoverable already found -> the rest of the level adds nothing
                    if (it >= nl || discovered + (long long)*(volatile unsigned long long*)&S->tdnew >= target) break;
                    const int c = list[it];
                    const int64_t rs = P.cell_scan_start[c];
                    const int nr = P.cell_nruns[c];
                    int nnew = 0;
                    for (int r = lane; r < nr; r += 64) nnew += run_push(V, X, tw, P.scan_pool[rs + r]);
                    for (int off = 32; off >= 1; off >>= 1) nnew += __shfl_xor(nnew, off);
                    if (lane == 0) {
                        runs_read += (unsigned long long)nr;
                        if (nnew) atomicAdd(&S->tdnew, (unsigned long long)nnew);
                    }
                }
                __syncthreads();
                if (tid == 0) { S->list_n = 0; S->item = 0; S->tdnew = 0; }
            }
            __syncthreads();
            // ---- level bookkeeping: count of X, next (expandable) frontier
            unsigned long long c_loc = 0, m_loc = 0;
            for (int i = tid; i < nt; i += DO_THREADS) {
                unsigned long long x = X[i];
                if (x) {
                    c_loc += (unsigned long long)__popcll(x);
                    if (P.radius != -1) x &= ~P.nonexp_tiles[i];
                    m_loc += (unsigned long long)__popcll(x);  // expandable part of the next frontier
                }
                F[i] = x;
                X[i] = 0ull;
            }
            for (int off = 32; off >= 1; off >>= 1) {
                c_loc += __shfl_xor(c_loc, off);
                m_loc += __shfl_xor(m_loc, off);
            }
            if (lane == 0 && c_loc) { atomicAdd(&S->cnt, c_loc); atomicAdd(&S->mass, m_loc); }
            if (P.nmp && (P.radius == -1 || level + 1 < P.radius)) {
                __syncthreads();   // the new level is in F and V
                merge_level_pass(P.mpairs, P.nmp, rows, tw, DO_THREADS, F, V, !GBM, P.seed_tiles, nullptr, nullptr, 0, 0,
                                 nullptr, level + 1, &S->mcorr, &S->mdisc, &S->mass);
                if (P.nmamb) {
                    __syncthreads();
                    merge_order_check(P.mamb, P.nmamb, rows, tw, DO_THREADS, F, V, !GBM, P.seed_tiles,
                                      P.mseen + (size_t)blockIdx.x * P.nmamb, (int32_t)src + 1, P.error, P.oflag, src);
                }
            }
            __syncthreads();
            const long long cnt = (long long)S->cnt, mass = (long long)S->mass;
            const long long mcorr = (long long)S->mcorr, mdisc = (long long)S->mdisc;
            __syncthreads();
            if (tid == 0) { S->cnt = 0; S->mass = 0; S->mcorr = 0; S->mdisc = 0; }
            if (cnt == 0) break;
            if (level + 1 >= P.maxlev) { overflow = true; break; }
            if (tid == 0) hist[level + 1] = (int)(cnt - mcorr);
            discovered += cnt + mdisc;
            m_u -= cnt + mdisc;
            m_f = mass;
            level++;
            nlev = level + 1;
            if (tid == 0) atomicAdd(&P.stats[bottom_up ? 3 : 4], 1ull);
            __syncthreads();
        }
        __syncthreads();
        if (overflow) {
            if (tid == 0) atomicOr(P.error, KERR_LEVELS);
            continue;
        }
        if (tid == 0) {
            long long tn, td;
            vga_measures(hist, nlev, o, tn, td);
            if (P.levels_out) {
                P.levels_out[src * 3 + 0] = tn;
                P.levels_out[src * 3 + 1] = td;
                P.levels_out[src * 3 + 2] = nlev;
            }
            atomicAdd(&P.stats[2], (unsigned long long)tn);
        }
        __syncthreads();
    }
    for (int off = 32; off >= 1; off >>= 1) {
        runs_read += __shfl_xor(runs_read, off);
        fail_cells += __shfl_xor(fail_cells, off);
        fail_runs += __shfl_xor(fail_runs, off);
    }
    if (lane == 0 && runs_read) atomicAdd(&P.stats[0], runs_read);
    if (lane == 0 && fail_cells) { atomicAdd(&P.stats[5], fail_cells); atomicAdd(&P.stats[6], fail_runs); }
}

// ---------------------------------------------------------------- symmetry / in-set corrections
// Bottom-up needs In(v) = {u filled : v in cells(u)} while it scans cells(v).  Per node we compare
// random-weighted sums HO(v) = sum_{w in cells(v)} s(w) and HI(v) = sum_{u : v in cells(u)} s(u)
// (64-bit wrap-around, s = splitmix64(cell), 0 for non-filled cells).  Every node involved in an
// asymmetric pair gets HO != HI except with probability 2^-64; those "special" nodes then get exact
// Extra (in-neighbours outside cells(v)) / Missing (cells(v) members that are not in-neighbours)
// lists built from their explicit cell sets.  Range sums / range adds along rows, columns and both
// diagonals make this O(runs).
// cell_weight, run_dir, dir_step and sym_run_scatter: common.hpp (makeGraph publishes the same scatter)

// lines along direction `dir`: start cell of line `line`
__device__ __forceinline__ bool line_start(int dir, int line, int cols, int rows, int& x, int& y) {
    if (dir == 0) { if (line >= rows) return false; x = 0; y = line; return true; }
    if (dir == 1) { if (line >= cols) return false; x = line; y = 0; return true; }
    if (line >= cols + rows - 1) return false;
    if (dir == 2) { if (line < rows) { x = 0; y = rows - 1 - line; } else { x = line - rows + 1; y = 0; } }
    else { if (line < rows) { x = 0; y = line; } else { x = line - rows + 1; y = rows - 1; } }
    return true;
}

// mode 0: in-place prefix sums of the filled-cell weights into P[dir][c]
// mode 1: in-place prefix sums of the difference arrays D[dir][c] (range adds -> values)
__global__ void sym_lines_kernel(int cols, int rows, const int32_t* cell_node, unsigned long long* arr, int mode) {
    const int64_t C = (int64_t)cols * rows;
    const int dir = blockIdx.y;
    const int line = blockIdx.x * blockDim.x + threadIdx.x;
    int x, y, dx, dy;
    if (!line_start(dir, line, cols, rows, x, y)) return;
    dir_step(dir, dx, dy);
    unsigned long long* A = arr + (int64_t)dir * C;
    unsigned long long acc = 0;
    for (; x >= 0 && x < cols && y >= 0 && y < rows; x += dx, y += dy) {
        const int64_t c = (int64_t)x * rows + y;
        if (mode == 0) acc += (cell_node[c] >= 0) ? cell_weight((unsigned long long)c) : 0ull;
        else acc += A[c];
        A[c] = acc;
    }
}

// HO per node (range sums over its runs) and range-add of s(u) into the difference arrays D
__global__ void sym_scatter_kernel(int cols, int rows, const int32_t* node_cell, int64_t n, const int64_t* node_run_start,
                                   const int32_t* node_nruns, const Run* pool, const unsigned long long* prefix,
                                   unsigned long long* diff, unsigned long long* ho) {
    const int64_t C = (int64_t)cols * rows;
    for (int64_t k = blockIdx.x; k < n; k += gridDim.x) {
        const int c = node_cell[k];
        const unsigned long long su = cell_weight((unsigned long long)c);
        const int64_t rs = node_run_start[k];
        const int nr = node_nruns[k];
        unsigned long long acc = 0;
        for (int r = threadIdx.x; r < nr; r += blockDim.x) acc += sym_run_scatter(pool[rs + r], su, cols, rows, prefix, diff);
        for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
        __shared__ unsigned long long red[16];
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long t = 0;
            for (int w = 0; w < (int)(blockDim.x >> 6); w++) t += red[w];
            ho[k] = t;
        }
        __syncthreads();
    }
}

// special nodes: HO != HI (HI = sum over the 4 directions of the range-added weights)
__global__ void sym_flag_kernel(int rows, const int32_t* node_cell, int64_t n, int64_t C, const unsigned long long* hi4,
                                const unsigned long long* ho, int* count, int32_t* list, int cap) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const int64_t c = node_cell[k];
    const unsigned long long hi = hi4[c] + hi4[C + c] + hi4[2 * C + c] + hi4[3 * C + c];
    if (hi != ho[k]) {
        const int pos = atomicAdd(count, 1);
        if (pos < cap) list[pos] = (int32_t)k;
    }
}

// Coverage counts: range-add 1 per run into int difference arrays (4 directions); after the line
// prefix pass a filled cell with a non-zero total appears in some run (it is in U_f).
__global__ void cov_scatter_kernel(int cols, int rows, int64_t n, const int64_t* node_run_start, const int32_t* node_nruns,
                                   const Run* pool, int* diff) {
    const int64_t C = (int64_t)cols * rows;
    for (int64_t k = blockIdx.x; k < n; k += gridDim.x) {
        const int64_t rs = node_run_start[k];
        const int nr = node_nruns[k];
        for (int r = threadIdx.x; r < nr; r += blockDim.x) {
            const Run ru = pool[rs + r];
            const int dir = run_dir(ru);
            int dx, dy;
            dir_step(dir, dx, dy);
            const int ex = ru.x1 + dx, ey = ru.y1 + dy;
            int* D = diff + (int64_t)dir * C;
            atomicAdd(&D[(int64_t)ru.x0 * rows + ru.y0], 1);
            if (ex >= 0 && ex < cols && ey >= 0 && ey < rows) atomicAdd(&D[(int64_t)ex * rows + ey], -1);
        }
    }
}
__global__ void cov_lines_kernel(int cols, int rows, int* arr) {
    const int64_t C = (int64_t)cols * rows;
    const int dir = blockIdx.y;
    const int line = blockIdx.x * blockDim.x + threadIdx.x;
    int x, y, dx, dy;
    if (!line_start(dir, line, cols, rows, x, y)) return;
    dir_step(dir, dx, dy);
    int* A = arr + (int64_t)dir * C;
    int acc = 0;
    for (; x >= 0 && x < cols && y >= 0 && y < rows; x += dx, y += dy) {
        const int64_t c = (int64_t)x * rows + y;
        acc += A[c];
        A[c] = acc;
    }
}
// U_f tiles (filled & covered), their complement, and the count
__global__ void cov_tiles_kernel(int cols, int rows, int tw, int th, const int32_t* cell_node, const int* cov,
                                 unsigned long long* uf, unsigned long long* notuf, unsigned long long* count) {
    const int64_t C = (int64_t)cols * rows;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= tw * th) return;
    const int tx = t % tw, ty = t / tw;
    unsigned long long w = 0;
    for (int b = 0; b < 64; b++) {
        const int x = tx * 8 + (b & 7), y = ty * 8 + (b >> 3);
        if (x >= cols || y >= rows) continue;
        const int64_t c = (int64_t)x * rows + y;
        if (cell_node[c] >= 0 && (cov[c] + cov[C + c] + cov[2 * C + c] + cov[3 * C + c]) > 0) w |= 1ull << b;
    }
    uf[t] = w;
    notuf[t] = ~w;
    if (w) atomicAdd(count, (unsigned long long)__popcll(w));
}

// U_f from the in-set hashes of the symmetry pass (hi4 = the four range-added weight arrays after
// their line prefix sums): a filled cell lies on some run iff some node sees it, i.e. its in-set is
// non-empty, i.e. HI = the sum of its in-neighbours' 64-bit weights is non-zero -- exact but for the
// 2^-64 chance per cell on which the symmetry certificate already rests.  Replaces the coverage
// counting pass (cov_scatter / cov_lines), one O(runs) scatter less per graph.
__global__ void uf_hi_tiles_kernel(int cols, int rows, int tw, int th, const int32_t* cell_node,
                                   const unsigned long long* hi4, unsigned long long* uf, unsigned long long* notuf,
                                   unsigned long long* count) {
    const int64_t C = (int64_t)cols * rows;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= tw * th) return;
    const int tx = t % tw, ty = t / tw;
    unsigned long long w = 0;
    for (int b = 0; b < 64; b++) {
        const int x = tx * 8 + (b & 7), y = ty * 8 + (b >> 3);
        if (x >= cols || y >= rows) continue;
        const int64_t c = (int64_t)x * rows + y;
        if (cell_node[c] >= 0 && (hi4[c] + hi4[C + c] + hi4[2 * C + c] + hi4[3 * C + c]) != 0ull) w |= 1ull << b;
    }
    uf[t] = w;
    notuf[t] = ~w;
    if (w) atomicAdd(count, (unsigned long long)__popcll(w));
}

// Scan pool: each node's runs in bottom-up scan order.  Runs are split into the 8 angular groups of
// 4 bins (bins 4g..4g+3), ordered longest-first inside a group (16 log2-length buckets), and the
// groups are interleaved round-robin: the first 8 entries are the longest run of each direction, so
// a cell hidden from the frontier in some directions still finds a hit early.  One workgroup per
// node; also fills the cell-indexed start / count arrays.
__global__ void scan_pool_kernel(int rows, const int32_t* node_cell, int64_t n, const int64_t* node_run_start,
                                 const int32_t* node_nruns, const int32_t* bin_nruns, const Run* pool,
                                 const int64_t* scan_start, Run* scan_pool, int64_t* cell_scan_start, int32_t* cell_nruns) {
    __shared__ int cnt[8][16], cur[8][16], ng[8], pre[33];
    for (int64_t k = blockIdx.x; k < n; k += gridDim.x) {
        const int64_t rs = node_run_start[k], ss = scan_start[k];
        const int nr = node_nruns[k];
        if (threadIdx.x < 128) cnt[threadIdx.x >> 4][threadIdx.x & 15] = 0;
        if (threadIdx.x < 32) pre[threadIdx.x + 1] = bin_nruns[k * 32 + threadIdx.x];
        if (threadIdx.x == 0) pre[0] = 0;
        __syncthreads();
        if (threadIdx.x == 0)
            for (int b = 1; b <= 32; b++) pre[b] += pre[b - 1];
        __syncthreads();
        for (int r = threadIdx.x; r < nr; r += blockDim.x) {
            int b = 0;
            while (pre[b + 1] <= r) b++;
            const Run ru = pool[rs + r];
            const int len = max(ru.x1 - ru.x0, max(ru.y1 - ru.y0, ru.y0 - ru.y1)) + 1;
            atomicAdd(&cnt[b >> 2][15 - min(15, 31 - __clz(len))], 1);
        }
        __syncthreads();
        if (threadIdx.x < 8) {
            const int g = threadIdx.x;
            int acc = 0;
            for (int b = 0; b < 16; b++) { cur[g][b] = acc; acc += cnt[g][b]; }
            ng[g] = acc;
        }
        if (threadIdx.x == 0) {
            const int c = node_cell[k];
            cell_scan_start[c] = ss;
            cell_nruns[c] = nr;
        }
        __syncthreads();
        for (int r = threadIdx.x; r < nr; r += blockDim.x) {
            int b = 0;
            while (pre[b + 1] <= r) b++;
            const int g = b >> 2;
            const Run ru = pool[rs + r];
            const int len = max(ru.x1 - ru.x0, max(ru.y1 - ru.y0, ru.y0 - ru.y1)) + 1;
            const int p = atomicAdd(&cur[g][15 - min(15, 31 - __clz(len))], 1);   // position inside group g
            int idx = 0;
            for (int h = 0; h < 8; h++) idx += min(p, ng[h]) + ((h < g && ng[h] > p) ? 1 : 0);
            scan_pool[ss + idx] = ru;
        }
        __syncthreads();
    }
}

// For each special node: the special cells inside cells(node) (explicit enumeration).
__global__ void sym_special_out_kernel(int rows, const int32_t* specials, int nspec, const int32_t* node_cell,
                                       const int32_t* cell_node, const uint8_t* is_special, const int64_t* node_run_start,
                                       const int32_t* node_nruns, const Run* pool, int32_t* out, int* out_n, int cap) {
    const int si = blockIdx.x;
    if (si >= nspec) return;
    const int k = specials[si];
    const int64_t rs = node_run_start[k];
    const int nr = node_nruns[k];
    for (int r = threadIdx.x; r < nr; r += blockDim.x) {
        const Run ru = pool[rs + r];
        int dx, dy;
        dir_step(run_dir(ru), dx, dy);
        int x = ru.x0, y = ru.y0;
        for (;;) {
            const int v = cell_node[(int64_t)x * rows + y];
            if (v >= 0 && is_special[v]) {
                const int pos = atomicAdd(&out_n[si], 1);
                if (pos < cap) out[(int64_t)si * cap + pos] = v;
            }
            if (x == ru.x1 && y == ru.y1) break;
            x += dx;
            y += dy;
        }
    }
}

} // namespace dmx
