// vga_tile.hip -- tile-resolved, direction-optimising VGA global BFS (+ the measures kernel and the
// preparation kernels it reads).
//
// Same result as VGAVisualGlobal::run (salalib/vgamodules/vgavisualglobal.cpp:23-216; set semantics as in
// vga_do.hip), organised so that one source costs O(tiles) rather than O(cells) of memory traffic:
//   * one 1024-thread workgroup per source (persistent grid); the frontier F is a bitmap of 8x8-cell tiles,
//     in LDS up to 1024 cells a side and in per-workgroup HBM above (FG, its line summaries stay in LDS);
//     the visited set V and the next level X live in per-workgroup HBM scratch, touched only for the tiles
//     the previous level listed as still holding an unvisited cell;
//   * level 1 is top-down: the source's runs are rasterised into F;
//   * later levels are bottom-up while Beamer's test on cell counts allows (valid because visibility is
//     symmetric; the few asymmetric nodes take exact in-set corrections, vga_do.hip prepare_symmetry):
//       A. tile level: the tile's common runs CR(t) (visible from every regular cell of the tile) against F;
//          one hit discovers all of the tile's unvisited regular cells;
//       B. a wave per remaining tile, lane = cell: the tile-to-tile rows (ttvis / ttany), then each cell's
//          first head runs and its hint (the run or partial-tile mask that last hit), then the other heads;
//       C. hard cells, a wave per cell: the tile-visibility rows (tvis / ftvis) give a certain hit or miss,
//          the partial-tile masks decide the rest exactly; without the masks (memory, grids above 1024 a
//          side) the cell's runs are scanned, with the tvis rows (and their summaries) as a miss certificate;
//   * top-down again when Beamer's test prefers it (small frontier); the bookkeeping publishes the
//     expandable part of X as the next F and rebuilds F's summaries.
// DESIGN.md section 2 has the measurements behind each choice, including the variants measured and dropped
// (phase-C prefix loaded with the row word, heads 4..7 loaded with the hint's operand, prefetching the next
// queue entry or hard-cell chunk, more masks in flight).
#include "common.hpp"

namespace dmx {

constexpr int KH = 8;        // head runs per cell (first KH entries of its scan order)
// heads and tile-common runs are ordered row / column runs first (1000^2: VGA 7.50 -> 6.11 s, phase A's
// clocks / 5.7: a diagonal run's test walks its tiles, 8 LDS reads a round trip)
constexpr int CRK = 4;       // tile-common runs per tile
constexpr int BEXT_DEFAULT = 0;   // scan-order runs past the KH heads phase B tests (final build: 0 -1.4 % vs 4, profiles/r3b_vga_env)
constexpr int VGA_HMAX = 64;  // levels kept per source by the tile kernel (deeper: vga_do)

struct VgaTileParams {
    int cols, rows, tw, th;
    const unsigned long long* seed_tiles;     // cells never discoverable (non-filled, outside U_f, padding)
    const unsigned long long* regular_tiles;  // U_f cells that are not special (asymmetric)
    const unsigned long long* nonexp_tiles;   // contextfilled odd cells (radius != -1)
    const Run* cr;                            // [nt][CRK] tile-common runs, longest first (x0 < 0: none)
    const Run* heads;                         // [KH][nt*64] tile-ordered head runs (x0 < 0: none)
    const int64_t* tscan_start;               // [nt*64] start in scan_pool (tile order)
    const int32_t* tnruns;                    // [nt*64]
    const Run* scan_pool;
    const unsigned long long* tvis;           // [nt*64][tvw] tiles seen by each cell, Fsr layout (null: off)
    const unsigned long long* ftvis;          // [nt*64][tvw] tiles whose every non-seed cell the cell sees (null: off)
    const unsigned long long* ttvis;          // [nt][tvw] AND of ftvis over the tile's regular cells (null: off)
    const unsigned long long* ttany;          // [nt][tvw] OR of tvis over the tile's regular cells
    const unsigned long long* pmask;          // partial-tile masks: per cell, the seen cells of each tile in
                                              // tvis & ~ftvis, in row-word then bit order (null: off)
    const int64_t* poff;                      // [nt*64 + 1] start of each cell's masks in pmask
    const uint16_t* ppre;                     // [nt*64][tvw] partial tiles of the cell before each row word
    int tvw;                                  // th * ceil(tw / 64)
    const unsigned long long* tvsum;          // [nt*64][ceil(tvw / 64)] non-zero row words (wide grids; null: off)
    const unsigned long long* tvnz;           // [nt*64][ceil(tvw / 64)] the same on grids up to 256 row words: phase C
                                              // loads only a hard cell's non-zero row words (null: off)
    const int32_t* node_cell;
    const int32_t* cell_node;
    const uint8_t* node_flags;
    const int64_t* node_run_start;
    const int32_t* node_nruns;
    const Run* pool;
    const int32_t* spec_index;
    const int32_t* extra_off;
    const int32_t* extra;
    const int32_t* missing_off;
    const int32_t* missing;
    int64_t src_begin, src_end;
    int radius, gates_only;
    int64_t uf_count;
    int alpha;
    int* work_counter;
    int nwork;                // work items (chunks)
    DmxCtl* ctl;              // host-mapped progress / cancel block (nullptr: none)
    int chunk;                // consecutive sources per work grab (neighbouring sources share hints)
    uint32_t* hint;           // [nt*64] what last hit for a recent source: the scan position of a run, or
                              // (bit 31) a partial-tile mask: tile << 16 | its slot in the cell's list (~0u:
                              // none); shared by all workgroups: a stale value only costs one test
    uint32_t* hint2;          // [VGA_H2][nt*64] (narrow grids with the masks) more hints: the fully seen tiles the
                              // cell's hint held before later hits replaced it, newest first
                              // (0x80000000 | tile << 16 | 0xFFFF), or ~0
    unsigned long long* hintw;// [nt*64] wide grids' mask hints (their tile index needs 16 bits): (tile + 1) << 32 |
                              // slot, 0 none (null below 1024 cells a side)
    unsigned long long* xg;   // per workgroup [2][nt]: V (visited) then X (next level)
    unsigned long long* fg;   // per workgroup [nt]: the frontier F (vga_tile_kernel<..., FG = true> only)
    int4* queue;              // per workgroup [nt]: (tile, 0, mask lo, mask hi)
    int32_t* list;            // per workgroup [2][nt*64]: hard cells / frontier cells, then phase-B2 cells
    int32_t* tlist;           // per workgroup [2][nt]: tiles holding an unvisited cell (built by one level's
                              // bookkeeping for the next level: phase A and the bookkeeping walk only them)
    int maxlev;
    // seed mode (visual step depth, vgavisualglobaldepth.cpp:23-77): one BFS from nseeds seed nodes
    // (level 0, always expanded); contextfilled odd cells are never expanded at later levels;
    // cell_level[tile id] receives the level of every cell reached (launch one source, one block)
    const int32_t* seeds;
    int nseeds;
    const int32_t* src_list;  // optional: work index i -> source node src_list[i] (multi-GPU interleaved shards)
    int32_t* cell_level;
    int bext;                 // phase-B runs after the heads (BEXT_DEFAULT)
    int crk;                  // tile-common runs tested in phase A (<= CRK)
    const int2* mpairs;       // [nmp] merge links (cell a, cell b), x-major (Point::m_merge; nullptr: none)
    int nmp;
    const int2* mamb;         // [nmamb] links with a context-filled odd end (that end first; merge_order_check)
    int nmamb;
    int32_t* mseen;           // per workgroup [nmamb] (merge_order_check)
    uint8_t* oflag;           // [N] sources whose result depends on the reference's pop order (merge_order_check)
    int32_t* hist_out;        // [N][VGA_HMAX] level histogram per source (measures: vga_measures_kernel)
    int32_t* nlev_out;        // [N] levels (0: source skipped)
    int* error;
    // Asymmetric mode (a graph re-read from a .graph file, whose 4-bit row shifts moved runs): the search runs on a
    // symmetric reference graph R (the structures above) with the frontier F limited to cells outside A, the nodes
    // whose runs differ from R's (plus R's own asymmetric nodes); A's frontier cells push the graph's actual runs
    // (apool) top-down instead.  Exact: every edge between two cells outside A is in both graphs and symmetric.
    const unsigned long long* asym_tiles;   // [nt] cells of A (null: off)
    const unsigned long long* asym_uf;      // [nt] cells on some run of R (the bottom-up candidates)
    const Run* apool;                       // the graph's own runs
    const int64_t* arun_start;
    const int32_t* anruns;
    int32_t* alist;                         // per workgroup [alist_cap]: A cells of the frontier (tile ids)
    int alist_cap;
    unsigned long long* stats;  // [0] runs tested, [2] cells reached, [3] BU levels, [4] TD levels,
                                // [5] hard cells without a hit, [6] their runs, [7] tiles resolved by CR,
                                // [8..12] phase clocks, [13] hard cells rejected by their tile-visibility row,
                                // [14] tile-visibility rows read, [1] phase-C hits, [15] phase-C runs,
                                // [16] phase-C hits certified by a fully seen frontier tile, [17] top-down clocks,
                                // [18] phase-B tiles, [19] phase-B cells, [20] phase-B tiles resolved by ttvis, [25] pruned by ttany
};

__device__ __forceinline__ int tile_id_of(int x, int y, int tw) {
    return (((y >> 3) * tw + (x >> 3)) << 6) | ((y & 7) << 3) | (x & 7);
}
__device__ __forceinline__ void xy_of_tile_id(int id, int tw, int& x, int& y) {
    const int t = id >> 6, b = id & 63;
    x = (t % tw) * 8 + (b & 7);
    y = (t / tw) * 8 + (b >> 3);
}

// The per-workgroup HBM scratch (V, X, queues, hints) is only ever touched by its own workgroup,
// so workgroup scope is enough for every atomic and every ordering point: the atomics stay in the
// XCD's L2 and the barriers need no L2 write-back (agent scope would bypass / flush the
// non-coherent per-XCD L2 on every level).
__device__ __forceinline__ unsigned long long ld_wg(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void or_wg(unsigned long long* p, unsigned long long v) {
    __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void sync_global() { __syncthreads(); }

// The n cells (x + i, y + dy*i) of a diagonal run that stay inside the tile of (x, y), as that
// tile's bit mask (bit (y&7)*8 + (x&7)); n is bounded by the tile edges and the run's end xe.
__device__ __forceinline__ unsigned long long diag_tile_mask(int x, int y, int dy, int xe, int& n) {
    const int lx = x & 7, ly = y & 7;
    n = min(min(8 - lx, dy > 0 ? 8 - ly : ly + 1), xe - x + 1);
    const int b0 = ly * 8 + lx;
    if (dy > 0) return (0x8040201008040201ull << b0) & (~0ull >> (63 - (b0 + 9 * (n - 1))));   // bits b0 + 9i
    const int first = b0 - 7 * (n - 1);                                                        // bits b0 - 7i
    const unsigned long long a = 0x0102040810204080ull;                                        // bits 7, 14, .., 56
    return (first >= 7 ? (a << (first - 7)) : (a >> (7 - first))) & (~0ull << first) & (~0ull >> (63 - b0));
}
// OR all cells of run `ru` into the tiled bitmap `bm` (LDS or HBM, atomic).
__device__ __forceinline__ void run_or(unsigned long long* bm, int tw, Run ru) {
    if (ru.y0 == ru.y1 && ru.x0 != ru.x1) {
        const int y = ru.y0, rowoff = (y >> 3) * tw, sh = (y & 7) * 8;
        for (int tx = ru.x0 >> 3; tx <= (ru.x1 >> 3); tx++) {
            const int lo = max((int)ru.x0, tx * 8) & 7, hi = min((int)ru.x1, tx * 8 + 7) & 7;
            or_wg(&bm[rowoff + tx], (unsigned long long)((0xFFu >> (7 - hi)) & (0xFFu << lo) & 0xFFu) << sh);
        }
    } else if (ru.x0 == ru.x1 && ru.y0 != ru.y1) {
        const int x = ru.x0, tx = x >> 3;
        const unsigned long long col = 0x0101010101010101ull << (x & 7);
        for (int ty = ru.y0 >> 3; ty <= (ru.y1 >> 3); ty++) {
            const int lo = max((int)ru.y0, ty * 8) & 7, hi = min((int)ru.y1, ty * 8 + 7) & 7;
            or_wg(&bm[ty * tw + tx], col & (~0ull >> (8 * (7 - hi))) & (~0ull << (8 * lo)));
        }
    } else {
        const int dy = (ru.y1 > ru.y0) ? 1 : -1;
        int x = ru.x0, y = ru.y0;
        while (x <= ru.x1) {
            int n;
            const unsigned long long m = diag_tile_mask(x, y, dy, ru.x1, n);
            or_wg(&bm[(y >> 3) * tw + (x >> 3)], m);
            x += n;
            y += dy * n;
        }
    }
}


// Run test against the LDS frontier with coarse occupancy summaries: Fsr (bit per tile, tile rows
// in row-major order) and Fsc (bit per tile, tile columns) give the tiles of the run that hold a
// frontier cell (a miss -- the common case when a cell's visible region lies in the source's
// shadow -- costs one or two summary reads).  The frontier words of those tiles are then read up to
// 8 at a time (independent LDS reads, OR-accumulated), so a long run through a dense frontier costs
// O(tiles / 8) dependent LDS round trips rather than O(tiles).
struct FView {
    const unsigned long long* F;
    const unsigned long long* Fsr;
    const unsigned long long* Fsc;
    const unsigned long long* RB;   // [th*8][wr]: bit tx of row y: tile (tx, y>>3) has a frontier cell in row y
    const unsigned long long* CB;   // [tw*8][wc]: bit ty of column x: tile (x>>3, ty) has one in column x
    int tw, wr, wc;
};
// attribution builds (scripts/gpu_vga_fetch.sh; off by default): row-word counters in phase C, phase C off,
// phase C without its mask loads
#ifndef VGA_ROWSTAT
#define VGA_ROWSTAT 0
#endif
#ifndef VGA_PHASEC_OFF
#define VGA_PHASEC_OFF 0
#endif
#ifndef VGA_PHASEC_ROWSONLY
#define VGA_PHASEC_ROWSONLY 0
#endif
#ifndef VGA_HINTS
#define VGA_HINTS 4          // hint slots a cell (narrow grids with the masks): the hint + VGA_HINTS - 1 fully seen
                             // tiles in hint2 (1000^2 VGA: 1 -> 3.858 s, 2 -> 3.684, 3 -> 3.568; on a later box
                             // 3 -> 3.688, 4 -> 3.513, 5 -> 3.553: profiles/r6_vga_hints_ab.jsonl)
#endif
#define VGA_H2 (VGA_HINTS - 1)   // slots of hint2: [VGA_H2][nt*64]
static_assert(VGA_HINTS >= 2, "hint2 holds at least one slot");
#ifndef VGA_TVNZ
#define VGA_TVNZ 0           // 1 = phase C loads only a hard cell's non-zero row words (row summaries tvnz)
#endif
#ifndef VGA_CCH
#define VGA_CCH 16           // phase C: hard-list entries a wave takes at once (1000^2 VGA: 8 -> 4.133 s, 16 -> 4.143, 32 -> 4.218)
#endif
#ifndef VGA_WIDE_PAIR
#define VGA_WIDE_PAIR 1      // wide grids: the mask test takes two row-summary groups a round
#endif
#ifndef VGA_WIDE_ROWPASS
#define VGA_WIDE_ROWPASS 0   // wide grids with masks: 1 = phase C row pass (2 cells a round) before the mask test (2000^2: 2.32 ms a source; 0: 2.17)
#endif

// A run as one 64-bit word: the runs a loop picks with a non-constant index are kept as separate words and
// chosen by selects (an indexed private array would live in scratch memory: a store and a load a lane per
// element and use, ~1 TB a launch at 1000^2 with the spills)
__device__ __forceinline__ Run run_of(unsigned long long w) {
    Run r;
    __builtin_memcpy(&r, &w, sizeof(Run));
    return r;
}
__device__ __forceinline__ unsigned long long run_word(const Run* p) { return *(const unsigned long long*)p; }

// Workgroup-shared scalars read from LDS after a barrier are the same in every lane: reading them through
// readfirstlane keeps them (and the level loop's counters built from them) in scalar registers instead of
// 64-bit VGPR pairs that the 128-VGPR budget spills around every level
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ long long uni64(unsigned long long v) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return (long long)(((unsigned long long)hi << 32) | lo);
}
// Tiles [t0, t1] of one summary line (bit per tile, one word per 64 tiles):
// OR of F[base + tx * stride] & (cell mask of tile tx), 8 frontier tiles per round.
template <bool VERT>
__device__ __forceinline__ bool line_hits(const unsigned long long* F, const unsigned long long* sum, int base, int stride,
                                          int t0, int t1, int a, int b, int sh) {
    const int w0 = t0 >> 6, w1 = t1 >> 6;
    for (int w = w0; w <= w1; w++) {
        unsigned long long m = sum[w];
        if (w == w0) m &= ~0ull << (t0 & 63);
        if (w == w1) m &= ~0ull >> (63 - (t1 & 63));
        while (m) {
            const int p = __ffsll((long long)m) - 1;
            unsigned long long acc = 0ull;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                if (p + j < 64 && ((m >> (p + j)) & 1ull)) {
                    const int tx = w * 64 + p + j;
                    const int lo = (tx == t0) ? a : 0, hi = (tx == t1) ? b : 7;
                    unsigned long long cm;
                    if (VERT) cm = (0x0101010101010101ull << sh) & (~0ull >> (8 * (7 - hi))) & (~0ull << (8 * lo));
                    else cm = (unsigned long long)((0xFFu >> (7 - hi)) & (0xFFu << lo) & 0xFFu) << sh;
                    acc |= F[base + tx * stride] & cm;
                }
            }
            if (acc) return true;
            m = (p + 8 >= 64) ? 0ull : (m & (~0ull << (p + 8)));
        }
    }
    return false;
}
// Diagonal run (Bin::make's single first-to-last span, ngraph.cpp:243-258): walked tile by tile;
// the run's cells inside one 8x8 tile are a shifted (anti-)diagonal bit pattern, so a tile costs
// one summary bit and at most one frontier word instead of up to 8 per-cell tests.
// The tile sequence of a run does not depend on the frontier, so the frontier words of 8 tiles are
// read per round (independent LDS reads, OR-accumulated): a run across the grid costs ~16 dependent
// LDS round trips instead of ~125.
__device__ __forceinline__ bool diag_hits(const FView& V, Run ru) {
    const int dy = (ru.y1 > ru.y0) ? 1 : -1;
    int x = ru.x0, y = ru.y0;
    while (x <= ru.x1) {
        unsigned long long acc = 0ull;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (x <= ru.x1) {
                int n;
                const unsigned long long m = diag_tile_mask(x, y, dy, ru.x1, n);
                acc |= V.F[(y >> 3) * V.tw + (x >> 3)] & m;
                x += n;
                y += dy * n;
            }
        }
        if (acc) return true;
    }
    return false;
}

// Line-resolved summaries (RB / CB): a run along one row (column) covers every cell of its interior
// tiles in that row (column), so a summary bit there is a hit; only the two end tiles need their
// frontier word.  At most 2 summary reads + 2 frontier reads per run on grids <= 1024 a side; wider lines
// (frontier in HBM, vga_tile_kernel<..., FG>) read the summary words between the ends as well.
__device__ __forceinline__ bool line_hits_rb(const unsigned long long* F, const unsigned long long* sum, int fbase, int fstride,
                                             int t0, int t1, unsigned long long m_first, unsigned long long m_last) {
    const int w0 = t0 >> 6, w1 = t1 >> 6;
    unsigned long long a = sum[w0] & (~0ull << (t0 & 63));
    unsigned long long b = 0ull;
    if (w1 == w0) a &= ~0ull >> (63 - (t1 & 63));
    else b = sum[w1] & (~0ull >> (63 - (t1 & 63)));
    const bool f0 = (a >> (t0 & 63)) & 1ull;
    const bool f1 = ((w1 == w0 ? a : b) >> (t1 & 63)) & 1ull;
    unsigned long long ia = a & ~(1ull << (t0 & 63)), ib = b;
    if (w1 == w0) ia &= ~(1ull << (t1 & 63));
    else ib &= ~(1ull << (t1 & 63));
    if (ia | ib) return true;   // an interior tile: its whole row (column) segment is on the run
    for (int w = w0 + 1; w < w1; w++)
        if (sum[w]) return true;
    if (!(f0 | f1)) return false;
    if (t0 == t1) return f0 && (F[fbase + t0 * fstride] & m_first & m_last);
    return (f0 && (F[fbase + t0 * fstride] & m_first)) || (f1 && (F[fbase + t1 * fstride] & m_last));
}
__device__ __forceinline__ bool run_hits_fs(const FView& V, Run ru) {
    if (V.RB && ru.y0 == ru.y1) {
        const int y = ru.y0, sh = (y & 7) * 8;
        return line_hits_rb(V.F, V.RB + y * V.wr, (y >> 3) * V.tw, 1, ru.x0 >> 3, ru.x1 >> 3,
                            (unsigned long long)((0xFFu << (ru.x0 & 7)) & 0xFFu) << sh,
                            (unsigned long long)(0xFFu >> (7 - (ru.x1 & 7))) << sh);
    }
    if (V.RB && ru.x0 == ru.x1) {
        const int x = ru.x0;
        const unsigned long long colm = 0x0101010101010101ull << (x & 7);
        return line_hits_rb(V.F, V.CB + x * V.wc, x >> 3, V.tw, ru.y0 >> 3, ru.y1 >> 3,
                            colm & (~0ull << (8 * (ru.y0 & 7))), colm & (~0ull >> (8 * (7 - (ru.y1 & 7)))));
    }
    if (ru.y0 == ru.y1) {   // horizontal (or a single cell): tile row ty, tiles x0>>3 .. x1>>3
        const int y = ru.y0, ty = y >> 3;
        return line_hits<false>(V.F, V.Fsr + ty * V.wr, ty * V.tw, 1, ru.x0 >> 3, ru.x1 >> 3, ru.x0 & 7, ru.x1 & 7,
                                (y & 7) * 8);
    } else if (ru.x0 == ru.x1) {   // vertical: tile column tx, tiles y0>>3 .. y1>>3
        const int x = ru.x0, tx = x >> 3;
        return line_hits<true>(V.F, V.Fsc + tx * V.wc, tx, V.tw, ru.y0 >> 3, ru.y1 >> 3, ru.y0 & 7, ru.y1 & 7, x & 7);
    } else {
        return diag_hits(V, ru);
    }
}

struct TileShared {
    int src, qn, hn, item, bn;
    int an, aitem;        // asymmetric mode: A cells listed for the next push, the push's work counter
    int tn[2];            // entries of the two unvisited-tile lists (level parity)
    int mpart;            // merge partner cell of the source (-1: none)
    unsigned long long cnt, mass;
    unsigned long long mcorr, mdisc;   // merge pass: pairs discovered together, partners of U_f joined
    long long m_f, m_u, disc, target;  // the level loop's state (in LDS: no VGPRs live across the levels)
};

// Next work item: one grid counter (progress and cancel ride on it).  Contiguous per-XCD ranges, so that an
// XCD's workgroups share their L2 on neighbouring sources, measured 1.1 % slower.
__device__ __forceinline__ int grab_work(DmxCtl* ctl, int* work_counter) {
    return ctl_poll(ctl, atomicAdd(work_counter, 1));
}

// Frontier cells on run `ru` (rare path: exact count for the asymmetric nodes).
__device__ __forceinline__ int run_count_f(const unsigned long long* F, int tw, Run ru) {
    int c = 0;
    if (ru.y0 == ru.y1) {
        const int y = ru.y0, ty = y >> 3, sh = (y & 7) * 8;
        for (int tx = ru.x0 >> 3; tx <= (ru.x1 >> 3); tx++) {
            const int lo = max((int)ru.x0, tx * 8) & 7, hi = min((int)ru.x1, tx * 8 + 7) & 7;
            c += __popcll(F[ty * tw + tx] & ((unsigned long long)((0xFFu >> (7 - hi)) & (0xFFu << lo) & 0xFFu) << sh));
        }
    } else if (ru.x0 == ru.x1) {
        const int x = ru.x0, tx = x >> 3;
        const unsigned long long colm = 0x0101010101010101ull << (x & 7);
        for (int ty = ru.y0 >> 3; ty <= (ru.y1 >> 3); ty++) {
            const int lo = max((int)ru.y0, ty * 8) & 7, hi = min((int)ru.y1, ty * 8 + 7) & 7;
            c += __popcll(F[ty * tw + tx] & colm & (~0ull >> (8 * (7 - hi))) & (~0ull << (8 * lo)));
        }
    } else {
        const int dy = (ru.y1 > ru.y0) ? 1 : -1;
        int y = ru.y0;
        for (int x = ru.x0; x <= ru.x1; x++, y += dy) c += (int)((F[(y >> 3) * tw + (x >> 3)] >> ((y & 7) * 8 + (x & 7))) & 1ull);
    }
    return c;
}
__device__ __forceinline__ bool cell_on_run(Run ru, int x, int y) {
    if (ru.y0 == ru.y1) return y == ru.y0 && x >= ru.x0 && x <= ru.x1;
    if (ru.x0 == ru.x1) return x == ru.x0 && y >= ru.y0 && y <= ru.y1;
    if (x < ru.x0 || x > ru.x1) return false;
    return y == ru.y0 + ((ru.y1 > ru.y0) ? 1 : -1) * (x - ru.x0);
}

// Exact bottom-up test for a node with asymmetric visibility (rare): hit iff some frontier cell u
// is an in-neighbour, i.e. u in Extra(v), or u in cells(v) and u not in Missing(v).  Whole wave:
// Extra first, then the tile-visibility prune, then the scan order 64 runs a step with the summary
// run test; a run that hits is confirmed unless every frontier cell on it is a Missing cell.
__device__ __forceinline__ bool special_hit(const VgaTileParams& P, const FView& FV, int id, int x, int y, int* nr_out) {
    const int lane = threadIdx.x & 63;
    const int tw = P.tw, rows = P.rows;
    const unsigned long long* F = FV.F;
    const int node = P.cell_node[x * rows + y];
    const int si = P.spec_index[node];
    const int64_t rs = P.tscan_start[id];
    const int nr = P.tnruns[id];
    const int e0 = P.extra_off[si], e1 = P.extra_off[si + 1];
    const int m0 = P.missing_off[si], m1 = P.missing_off[si + 1];
    *nr_out = nr;
    bool h = false;
    for (int j = e0 + lane; j < e1; j += 64) {
        const int uc = P.node_cell[P.extra[j]];
        const int ux = uc / rows, uy = uc % rows;
        if (F[(uy >> 3) * tw + (ux >> 3)] & (1ull << ((uy & 7) * 8 + (ux & 7)))) h = true;
    }
    if (__ballot(h) != 0ull) return true;
    if (P.tvis) {
        const unsigned long long* tv = P.tvis + (size_t)id * P.tvw;
        unsigned long long ta = 0ull;
        for (int j = 0; j * 64 < P.tvw; j++) {
            const int w = j * 64 + lane;
            if (w < P.tvw) ta |= tv[w] & FV.Fsr[w];
        }
        if (__ballot(ta != 0ull) == 0ull) return false;
    }
    for (int base = 0; base < nr; base += 64) {
        const int r = base + lane;
        if (r < nr) {
            const Run ru = P.scan_pool[rs + r];
            if (run_hits_fs(FV, ru)) {
                int nm = 0;   // Missing cells on this run that are in the frontier
                for (int j = m0; j < m1; j++) {
                    const int mc = P.node_cell[P.missing[j]];
                    const int mx = mc / rows, my = mc % rows;
                    if (cell_on_run(ru, mx, my) && ((F[(my >> 3) * tw + (mx >> 3)] >> ((my & 7) * 8 + (mx & 7))) & 1ull)) nm++;
                }
                h = nm == 0 || run_count_f(F, tw, ru) > nm;
            }
        }
        if (__ballot(h) != 0ull) return true;
    }
    return false;
}

// The in-set corrections of an asymmetric node v (whole wave): whether a frontier cell is in Extra(v) (an
// in-neighbour outside cells(v): a hit), and how many frontier cells are in Missing(v) (cells of v that are not
// in-neighbours; Missing(v) is a subset of cells(v), built in prepare_symmetry).  With none of the latter,
// v's in-set meets F iff cells(v) does, which the partial-tile masks decide as for a regular cell.
__device__ __forceinline__ bool special_extra_hit(const VgaTileParams& P, const unsigned long long* F, int node,
                                                  int* nmiss_f) {
    const int lane = threadIdx.x & 63;
    const int tw = P.tw, rows = P.rows;
    const int si = P.spec_index[node];
    const int e0 = P.extra_off[si], e1 = P.extra_off[si + 1];
    const int m0 = P.missing_off[si], m1 = P.missing_off[si + 1];
    bool h = false;
    int nm = 0;
    for (int j = e0 + lane; j < e1; j += 64) {
        const int uc = P.node_cell[P.extra[j]];
        const int ux = uc / rows, uy = uc % rows;
        if (F[(uy >> 3) * tw + (ux >> 3)] & (1ull << ((uy & 7) * 8 + (ux & 7)))) h = true;
    }
    for (int j = m0 + lane; j < m1; j += 64) {
        const int mc = P.node_cell[P.missing[j]];
        const int mx = mc / rows, my = mc % rows;
        if ((F[(my >> 3) * tw + (mx >> 3)] >> ((my & 7) * 8 + (mx & 7))) & 1ull) nm++;
    }
    for (int off = 32; off >= 1; off >>= 1) nm += __shfl_xor(nm, off);
    *nmiss_f = nm;
    return __ballot(h) != 0ull;
}

__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int u = __shfl_up(v, off, 64);
        if (lane >= off) v += u;
    }
    return v;
}

// Exact bottom-up test of a regular cell from its tile-visibility rows and partial-tile masks (whole
// wave): the cell sees a frontier cell iff a frontier tile lies under its full-visibility row, or the
// frontier word of one of its partially seen tiles meets that tile's mask.  The cell's visible set is
// its out-set; a regular cell's in-set is the same set, so this is the bottom-up test with no run
// scan.  Phase C calls it only for cells whose rows left the answer open (no frontier tile under the
// full row, some under the any row), so only the partial tiles holding a frontier cell are tested.
// Lane `lane` owns row words lane + 64k and reads them only under a frontier tile row (Fsr), as the
// row test before it did (L2 hits); a mask's position is the word's partial-tile prefix (ppre) plus
// the partial bits before it in the word (the order tile_pmask_kernel writes them in).  Up to 4 masks
// a lane are in flight per round.
__device__ __forceinline__ bool pmask_hit(const VgaTileParams& P, const unsigned long long* F,
                                          const unsigned long long* Fsr, int id, unsigned& nload, uint32_t* Hn) {
    const int lane = threadIdx.x & 63;
    const int tvw = P.tvw, tw = P.tw, wr = (P.tw + 63) / 64;
    const size_t row = (size_t)id * tvw;
    const unsigned long long* pm = P.pmask + P.poff[id];
#pragma unroll 1
    for (int k = 0; k * 64 < tvw; k++) {
        const int w = k * 64 + lane;
        const unsigned long long fs = w < tvw ? Fsr[w] : 0ull;
        unsigned long long pw = 0ull, cw = 0ull;
        int base = 0;
        if (fs) {
            pw = P.tvis[row + w] & ~P.ftvis[row + w];
            cw = pw & fs;
            if (cw) base = P.ppre[row + w];
        }
        const int trow = (w / wr) * tw + (w % wr) * 64;
        while (__ballot(cw != 0ull) != 0ull) {
            unsigned long long mk[4];
            int tl[4], sl[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                tl[j] = -1;
                if (cw) {
                    const int b = __ffsll((long long)cw) - 1;
                    cw &= cw - 1;
                    tl[j] = trow + b;
                    sl[j] = base + __popcll(pw & ((1ull << b) - 1ull));
                    mk[j] = pm[sl[j]];
                    nload++;
                }
            }
            int hj = -1;
#pragma unroll
            for (int j = 3; j >= 0; j--)
                if (tl[j] >= 0 && (F[tl[j]] & mk[j])) hj = j;
            const unsigned long long hb = __ballot(hj >= 0);
            if (hb != 0ull) {
                // the next source's phase B tests this tile's mask first (a hint, like a run position)
                if (lane == __ffsll((long long)hb) - 1) {
                    const int j = hj;
                    int t = tl[0], q = sl[0];
                    if (j == 1) { t = tl[1]; q = sl[1]; }
                    if (j == 2) { t = tl[2]; q = sl[2]; }
                    if (j == 3) { t = tl[3]; q = sl[3]; }
                    Hn[id] = 0x80000000u | ((uint32_t)t << 16) | (uint32_t)q;
                }
                return true;
            }
        }
    }
    return false;
}

// A hit replaced the cell's hint `hold`: a fully seen tile moves to the front of hint2, whose slots shift down
// (h2old: the slots before the last, loaded with the cell's row words).  One lane writes.
__device__ __forceinline__ void hint2_push(const VgaTileParams& P, int id, uint32_t hold, const uint32_t* h2old) {
    const size_t stride = (size_t)P.tw * P.th * 64;
#pragma unroll
    for (int k = 0; k + 1 < VGA_H2; k++)
        if (h2old[k] == hold) return;   // already held: keep the order
#pragma unroll
    for (int k = VGA_H2 - 1; k >= 1; k--) P.hint2[(size_t)k * stride + id] = h2old[k - 1];
    P.hint2[id] = hold;
}

// C_FUSED: the row test and the mask test in one pass per cell (no separate row-test pass over the chunk):
// the 4 row words of tvis and ftvis a lane owns are loaded together, a frontier tile under the full row is a
// certain hit, none under the partial bits a certain miss, else the masks of the partial frontier tiles.
__device__ __forceinline__ bool pmask_hit_fused(const VgaTileParams& P, const unsigned long long* F,
                                                const unsigned long long* Fsr, int id, unsigned& nload, uint32_t* Hn,
                                                int& how, unsigned nzb = 0xFu, unsigned* rstat = nullptr) {
    const int lane = threadIdx.x & 63;
    const int tvw = P.tvw, tw = P.tw, wr = (P.tw + 63) / 64;
    const size_t row = (size_t)id * tvw;
    unsigned long long pw[4], cw[4];
    int base[4];
    bool cert = false;
    int ct = -1;   // a frontier tile the cell sees completely (the lane's first): k << 6 | bit
    // the hint a hit here replaces: a fully seen tile moves to the second hint (loaded with the rows)
    const uint32_t hold = P.hint2 ? Hn[id] : 0xFFFFFFFFu;
    uint32_t h2old[VGA_H2 > 1 ? VGA_H2 - 1 : 1];   // the slots that shift down when the hint moves into hint2
#pragma unroll
    for (int k = 0; k + 1 < VGA_H2; k++) h2old[k] = P.hint2 ? P.hint2[(size_t)k * P.tw * P.th * 64 + id] : 0xFFFFFFFFu;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int w = k * 64 + lane;
        const unsigned long long fs = w < tvw ? Fsr[w] : 0ull;
        unsigned long long t = 0ull, f = 0ull;
        base[k] = 0;
        if (fs && ((nzb >> k) & 1u)) {   // nzb: the lane's row words that are non-zero (tvnz; ftvis lies in tvis)
            t = P.tvis[row + w];
            f = P.ftvis[row + w];
        }
        if (ct < 0 && (f & fs) != 0ull) ct = (k << 6) | (__ffsll((long long)(f & fs)) - 1);
        cert |= (f & fs) != 0ull;
        pw[k] = t & ~f;
        cw[k] = pw[k] & fs;
#if VGA_ROWSTAT
        if (rstat) {   // diagnostic build: row words loaded (per array), zero in tvis, zero in ftvis
            rstat[0] += __popcll(__ballot(fs != 0ull && ((nzb >> k) & 1u)));
            rstat[1] += __popcll(__ballot(fs != 0ull && t == 0ull));
            rstat[2] += __popcll(__ballot(fs != 0ull && f == 0ull));
        }
#endif
    }
    if (const unsigned long long cb = __ballot(cert)) {
        // the next source's phase B tests that tile first (slot 0xFFFF: the whole tile, no mask)
        if (lane == __ffsll((long long)cb) - 1) {
            const int w = (ct >> 6) * 64 + lane;
            const int t = (w / wr) * tw + (w % wr) * 64 + (ct & 63);
            const uint32_t hnew = 0x80000000u | ((uint32_t)t << 16) | 0xFFFFu;
            if (P.hint2 && (hold & 0x8000FFFFu) == 0x8000FFFFu && hold != 0xFFFFFFFFu && hold != hnew) {
                hint2_push(P, id, hold, h2old);
            }
            Hn[id] = hnew;
        }
        how = 1;
        return true;
    }
    if (__ballot((cw[0] | cw[1] | cw[2] | cw[3]) != 0ull) == 0ull) { how = 2; return false; }
    how = 0;
#if VGA_PHASEC_ROWSONLY
    return false;   // attribution build: no mask loads (results differ)
#endif
#pragma unroll
    for (int k = 0; k < 4; k++) base[k] = cw[k] ? (int)P.ppre[row + k * 64 + lane] : 0;
    const unsigned long long* pm = P.pmask + P.poff[id];
#pragma unroll 1
    for (int k = 0; k < 4; k++) {
        const int w = k * 64 + lane;
        const int trow = (w / wr) * tw + (w % wr) * 64;
        unsigned long long c = cw[k];
        const unsigned long long p = pw[k];
        const int bk = base[k];
        while (__ballot(c != 0ull) != 0ull) {
            constexpr int NM = 4;   // masks a lane keeps in flight (2: +1 %, 8: +34 %, round 4)
            unsigned long long mk[NM];
            int tl[NM], sl[NM];
#pragma unroll
            for (int j = 0; j < NM; j++) {
                tl[j] = -1;
                if (c) {
                    const int b = __ffsll((long long)c) - 1;
                    c &= c - 1;
                    tl[j] = trow + b;
                    sl[j] = bk + __popcll(p & ((1ull << b) - 1ull));
                    mk[j] = pm[sl[j]];
                    nload++;
                }
            }
            int hj = -1, ht = 0, hq = 0;
#pragma unroll
            for (int j = NM - 1; j >= 0; j--)
                if (tl[j] >= 0 && (F[tl[j]] & mk[j])) { hj = j; ht = tl[j]; hq = sl[j]; }
            const unsigned long long hb = __ballot(hj >= 0);
            if (hb != 0ull) {
                if (lane == __ffsll((long long)hb) - 1) {
                    if (P.hint2 && (hold & 0x8000FFFFu) == 0x8000FFFFu && hold != 0xFFFFFFFFu) {
                        hint2_push(P, id, hold, h2old);
                    }
                    Hn[id] = 0x80000000u | ((uint32_t)ht << 16) | (uint32_t)hq;
                }
                return true;
            }
        }
    }
    return false;
}

// The exact test on wide grids (tvw > 256 row words, row summaries tvsum), as pmask_hit_fused: a frontier tile
// under the full-visibility row is a hit, else the masks of the partial frontier tiles decide.  Lane `lane`
// takes the row words k*64 + lane whose summary bit is set (the cell's non-zero words) under a frontier tile
// row; a mask's position is ppre (the word's partial prefix) plus the partial bits before it.  (Regular cells
// come here after phase C's row pass found no certain hit; special nodes with no Missing cell in the frontier
// come directly.)  A mask that hits is recorded in hintw (the next source's phase B tests it first).
__device__ __forceinline__ bool pmask_hit_wide(const VgaTileParams& P, const unsigned long long* F,
                                               const unsigned long long* Fsr, int id, unsigned& nload) {
    const int lane = threadIdx.x & 63;
    const int tvw = P.tvw, tw = P.tw, wr = (P.tw + 63) / 64, tvsw = (tvw + 63) / 64;
    const size_t row = (size_t)id * tvw;
    const unsigned long long sm = lane < tvsw ? P.tvsum[(size_t)id * tvsw + lane] : 0ull;
    const unsigned long long* pm = P.pmask + P.poff[id];
    auto sum_word = [&](int k) -> unsigned long long {
        return (unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)sm, k) |
               ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)(sm >> 32), k) << 32);
    };
    // the masks of one group's partial frontier tiles, NM a lane in flight; a hit is recorded as a hint
    auto mask_group = [&](unsigned long long c, unsigned long long p, int bk, int w) -> bool {
        const int trow = (w / wr) * tw + (w % wr) * 64;
        while (__ballot(c != 0ull) != 0ull) {
            constexpr int NM = 4;
            unsigned long long mk[NM];
            int tl[NM], sl[NM];
#pragma unroll
            for (int j = 0; j < NM; j++) {
                tl[j] = -1;
                if (c) {
                    const int b = __ffsll((long long)c) - 1;
                    c &= c - 1;
                    tl[j] = trow + b;
                    sl[j] = bk + __popcll(p & ((1ull << b) - 1ull));
                    mk[j] = pm[sl[j]];
                    nload++;
                }
            }
            int ht = -1, hq = 0;
#pragma unroll
            for (int j = NM - 1; j >= 0; j--)
                if (tl[j] >= 0 && (F[tl[j]] & mk[j])) { ht = tl[j]; hq = sl[j]; }
            const unsigned long long hb = __ballot(ht >= 0);
            if (hb != 0ull) {
                if (P.hintw && lane == __ffsll((long long)hb) - 1)
                    P.hintw[id] = ((unsigned long long)(ht + 1) << 32) | (unsigned)hq;
                return true;
            }
        }
        return false;
    };
#if VGA_WIDE_PAIR
    // two summary groups a round: their row-word loads are independent, so they overlap
#pragma unroll 1
    for (int k = 0; k < tvsw; k += 2) {
        const unsigned long long s0 = sum_word(k), s1 = k + 1 < tvsw ? sum_word(k + 1) : 0ull;
        if ((s0 | s1) == 0ull) continue;
        const int w0 = k * 64 + lane, w1 = w0 + 64;
        const unsigned long long fs0 = ((s0 >> lane) & 1ull) ? Fsr[w0] : 0ull;
        const unsigned long long fs1 = ((s1 >> lane) & 1ull) ? Fsr[w1] : 0ull;
        unsigned long long f0 = 0ull, t0 = 0ull, f1 = 0ull, t1 = 0ull;
        if (fs0) { f0 = P.ftvis[row + w0]; t0 = P.tvis[row + w0]; }
        if (fs1) { f1 = P.ftvis[row + w1]; t1 = P.tvis[row + w1]; }
        if (__ballot(((f0 & fs0) | (f1 & fs1)) != 0ull) != 0ull) return true;
        const unsigned long long p0 = t0 & ~f0, c0 = p0 & fs0, p1 = t1 & ~f1, c1 = p1 & fs1;
        const int b0 = c0 ? (int)P.ppre[row + w0] : 0, b1 = c1 ? (int)P.ppre[row + w1] : 0;
        if (mask_group(c0, p0, b0, w0)) return true;
        if (mask_group(c1, p1, b1, w1)) return true;
    }
#else
#pragma unroll 1
    for (int k = 0; k < tvsw; k++) {
        const unsigned long long s = sum_word(k);
        if (s == 0ull) continue;
        const int w = k * 64 + lane;
        unsigned long long p = 0ull, c = 0ull;
        int bk = 0;
        bool cert = false;
        if ((s >> lane) & 1ull) {
            const unsigned long long fs = Fsr[w];
            if (fs) {
                const unsigned long long f = P.ftvis[row + w];
                cert = (f & fs) != 0ull;
                p = P.tvis[row + w] & ~f;
                c = p & fs;
                if (c) bk = P.ppre[row + w];
            }
        }
        if (__ballot(cert) != 0ull) return true;
        if (mask_group(c, p, bk, w)) return true;
    }
#endif
    return false;
}

// V (visited) and X (next level) are per-workgroup bitmaps in HBM (they stay in the L2/MALL; a
// source touches each word a few times), F (frontier, read by every run test) is in LDS.
// SPECIAL = false: the graph has no asymmetric nodes (every U_f cell is regular), no exact path.
// RBM: line-resolved summaries RB / CB in LDS (replace Fsc; need ~32 KB more LDS, grids <= ~1010^2).
// FG: grids whose frontier bitmap does not fit the LDS (above 1024 cells a side): F is a per-workgroup
// bitmap in HBM like V and X, and the LDS holds only its summaries (Fsr and RB / CB: 136 KB at 2000^2),
// so a row or column run still costs its summary words plus at most 2 frontier words.
template <int NT, bool SPECIAL, bool RBM, bool FG>
__global__ void __launch_bounds__(NT) vga_tile_kernel(const VgaTileParams* __restrict__ PP) {
    const DMX_CONST_AS VgaTileParams& P = const_params(PP);
    extern __shared__ __attribute__((aligned(16))) unsigned long long tile_smem[];
    __shared__ TileShared S;
    constexpr int NW = NT / 64;
    const int nt = P.tw * P.th;
    const int wr = (P.tw + 63) / 64, wc = (P.th + 63) / 64;
    const int nfs = RBM ? P.th * wr : P.th * wr + P.tw * wc;   // summary words rebuilt by atomics per level
    unsigned long long* F = FG ? P.fg + (size_t)blockIdx.x * nt : tile_smem;
    unsigned long long* Fsr = FG ? tile_smem : F + nt;   // [th][wr]
    unsigned long long* Fsc = Fsr + P.th * wr;  // [tw][wc] (!RBM)
    unsigned long long* RB = Fsr + P.th * wr;   // [th*8][wr] (RBM)
    unsigned long long* CB = RB + P.th * 8 * wr; // [tw*8][wc] (RBM)
    int* hist = (int*)(RBM ? (CB + P.tw * 8 * wc) : (Fsc + P.tw * wc));
    FView FV;
    FV.F = F; FV.Fsr = Fsr; FV.Fsc = RBM ? nullptr : Fsc; FV.tw = P.tw; FV.wr = wr; FV.wc = wc;
    FV.RB = RBM ? RB : nullptr;
    FV.CB = RBM ? CB : nullptr;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tw = P.tw, rows = P.rows;
    unsigned long long* Vg = P.xg + (size_t)blockIdx.x * 2 * nt;
    unsigned long long* Xg = Vg + nt;
    int4* Q = P.queue + (size_t)blockIdx.x * nt;
    int32_t* L = P.list + (size_t)blockIdx.x * nt * 64 * 2;
    int32_t* TL = P.tlist + (size_t)blockIdx.x * nt * 2;
    const size_t hstride = (size_t)nt * 64;
    // work counters live in LDS (flushed to P.stats at exit) so they cost no registers: a 1024-thread
    // workgroup has 128 VGPRs a lane and every spill is a scratch round trip
    __shared__ unsigned long long SC[32];
#define ST(k, v) atomicAdd(&SC[k], (unsigned long long)(v))
    unsigned rt = 0;                  // runs tested by this lane (flushed per source)
    unsigned long long tmark = 0;     // leader-thread phase clock
    for (int i = tid; i < 32; i += NT) SC[i] = 0ull;

    uint32_t* Hn = P.hint;
    if (tid == 0) {
        S.qn = 0; S.hn = 0; S.item = 0; S.bn = 0; S.cnt = 0; S.mass = 0; S.src = -1;
        S.mpart = -1; S.mcorr = 0; S.mdisc = 0;
        S.an = 0; S.aitem = 0;
    }
    int64_t chunk_end = 0;
    int64_t src = -1;
    for (;;) {
        // sources are taken in chunks of consecutive (spatially adjacent) nodes, whose BFSs hit
        // through the same runs: the hint array carries that knowledge from one source to the next
        if (src + 1 >= chunk_end) {
            __syncthreads();
            if (tid == 0) S.src = grab_work(P.ctl, P.work_counter);
            __syncthreads();
            src = P.src_begin + (int64_t)uni(S.src) * P.chunk;
            chunk_end = min(src + (int64_t)P.chunk, P.src_end);
        } else {
            src++;
        }
        if (src >= P.src_end) break;
        const int64_t node = P.src_list ? (int64_t)P.src_list[src] : src;   // the source node
        const bool seeded = P.nseeds > 0;
        const int scell = P.node_cell[seeded ? P.seeds[0] : node];
        const int sx = scell / rows, sy = scell % rows;
        // VGAVisualGlobal::run: context-filled odd sources and gates_only are skipped (:72-75)
        if (!seeded && (((P.node_flags[node] & 1) && !((sx % 2) == 0 && (sy % 2) == 0)) || P.gates_only)) {
            if (tid == 0) P.nlev_out[node] = 0;
            continue;
        }
        const int stile = (sy >> 3) * tw + (sx >> 3);
        const unsigned long long sbit = 1ull << ((sy & 7) * 8 + (sx & 7));
        for (int t = tid; t < nt; t += NT) {
            Vg[t] = P.seed_tiles[t] | (t == stile ? sbit : 0ull);
            Xg[t] = 0ull;
            F[t] = 0ull;
        }
        for (int i = tid; i < VGA_HMAX; i += NT) hist[i] = 0;
        long long n_in_uf = (P.seed_tiles[stile] & sbit) ? 0 : 1;
        if (seeded) {
            // every seed is visited at level 0; count those inside U_f for the early exit
            __syncthreads();
            for (int i = tid; i < P.nseeds; i += NT) {
                const int c = P.node_cell[P.seeds[i]];
                const int x = c / rows, y = c % rows;
                const int t = (y >> 3) * tw + (x >> 3);
                const unsigned long long b = 1ull << ((y & 7) * 8 + (x & 7));
                if (!(P.seed_tiles[t] & b) && !(t == stile && b == sbit)) atomicAdd(&S.cnt, 1ull);   // seeds[0] counted above
                or_wg(&Vg[t], b);
            }
            __syncthreads();
            n_in_uf += uni64(S.cnt);
            __syncthreads();
            if (tid == 0) S.cnt = 0;
        }
        // the source's merge partner is extracted at level 0 and never counted (vgavisualglobal.cpp:113-122);
        // in seed mode the host lists the seeds' partners as seeds (they take level 0)
        int64_t spart = -1;
        if (P.nmp && !seeded) {
            __syncthreads();
            for (int i = tid; i < P.nmp; i += NT) {
                const int2 pr = P.mpairs[i];
                if (pr.x == scell) S.mpart = pr.y;
                else if (pr.y == scell) S.mpart = pr.x;
            }
            __syncthreads();
            const int pc = uni(S.mpart);
            if (pc >= 0) {
                spart = P.cell_node[pc];
                const int px = pc / rows, py = pc % rows;
                const int pt = (py >> 3) * tw + (px >> 3);
                const unsigned long long pb = 1ull << ((py & 7) * 8 + (px & 7));
                if (tid == 0) or_wg(&Vg[pt], pb);
                if (!(P.seed_tiles[pt] & pb)) n_in_uf++;
            }
            __syncthreads();
            if (tid == 0) S.mpart = -1;
        }
        int level = 0, nlev = 1;
        bool overflow = false;
        if (tid == 0) {
            S.tn[0] = 0; S.tn[1] = 0;
            S.an = 0; S.aitem = 0;   // (a search that stopped at its radius leaves A cells listed)
            S.target = P.uf_count - n_in_uf;
            S.m_f = seeded ? P.nseeds : (spart >= 0 ? 2 : 1);
            S.m_u = S.target;
            S.disc = 0;
        }
        __syncthreads();
        if (tid == 0) hist[0] = seeded ? P.nseeds : 1;
        for (;;) {
            if (P.radius != -1 && level >= P.radius) break;
            if (uni64(S.disc) >= uni64(S.target)) break;
            const bool bottom_up = level > 0 && (uni64(S.m_f) * (long long)P.alpha > uni64(S.m_u));
            tmark = __builtin_amdgcn_s_memtime();
            if (level == 0) {
                // ---- level 1: rasterise the source's runs (top-down from {s}, or from every seed)
                for (int i = 0; i < (seeded ? P.nseeds : (spart >= 0 ? 2 : 1)); i++) {
                    const int64_t sn = seeded ? P.seeds[i] : (i == 0 ? node : spart);
                    // (asymmetric mode: a source in A sees along the graph's own runs)
                    const bool own = P.asym_tiles && i == 0 && !seeded && (P.asym_tiles[stile] & sbit);
                    const int64_t rs = own ? P.arun_start[sn] : P.node_run_start[sn];
                    const int nr = own ? P.anruns[sn] : P.node_nruns[sn];
                    const Run* pl = own ? P.apool : P.pool;
                    for (int r = tid; r < nr; r += NT) run_or(F, tw, pl[rs + r]);
                    if (tid < nr) rt += (unsigned)((nr - tid + NT - 1) / NT);
                }
                sync_global();
                for (int t = tid; t < nt; t += NT) Xg[t] = F[t] & ~Vg[t];
                if (tid == 0) { const unsigned long long n = __builtin_amdgcn_s_memtime(); ST(8, n - tmark); tmark = n; }
            } else if (bottom_up) {
                // ---- A: tile-common runs
                // only the tiles the previous level's bookkeeping listed can hold an unvisited cell
                const int32_t* TLc = TL + (level & 1) * nt;
                const int ntl = uni(S.tn[level & 1]);
                for (int t0 = 0; t0 < ntl; t0 += NT) {
                    const int t = t0 + tid < ntl ? TLc[t0 + tid] : nt;
                    unsigned long long U = 0ull, rg = ~0ull;
                    if (t < nt) {
                        // V, the regular mask and the CRK common runs in one round trip
                        static_assert(CRK == 4, "phase A keeps the common runs in four words");
                        const unsigned long long c0 = run_word(P.cr + CRK * t), c1 = run_word(P.cr + CRK * t + 1),
                                                 c2 = run_word(P.cr + CRK * t + 2), c3 = run_word(P.cr + CRK * t + 3);
                        U = ~Vg[t];
                        if (P.asym_tiles) U &= P.asym_uf[t];   // (cells off R's runs: only A pushes reach them)
                        rg = P.regular_tiles[t];
                        const unsigned long long R = U & rg;
                        if (R) {
// B_ORDER: the hint's operand is loaded before the head tests and tested after them (-0.7 %)
// RB_INC: line summaries set per published tile with LDS atomics instead of rebuilt from F (measured
// slower: bookkeeping clocks x1.9, contention on the summary words of a tile row)
// BEXT_NODIAG: phase B's extra run tests skip diagonal runs (a cell that misses then goes to phase C's exact
// mask test): 6.10 -> 5.62 s at 1000^2.  RB8: the line summaries rebuilt one F word read per tile (-0.05 s)
// C_FUSED: phase C's row test and mask test in one pass per cell (1000^2: VGA 5.57 -> 5.11 s)
                            bool hit = false;
#pragma unroll 1
                            for (int j = 0; j < CRK; j++) {
                                const Run cj = run_of(j == 0 ? c0 : j == 1 ? c1 : j == 2 ? c2 : c3);
                                if (!hit && j < P.crk && cj.x0 >= 0) {
                                    rt++;
                                    hit = run_hits_fs(FV, cj);
                                }
                            }
                            if (hit) { Xg[t] = R; U &= ~R; ST(7, 1); }   // (X holds nothing else yet: one thread a tile)
                        }
                    }
                    const unsigned long long want = __ballot(U != 0ull);
                    if (want) {
                        int base = 0;
                        if (lane == 0) base = atomicAdd(&S.qn, __popcll(want));
                        base = __shfl(base, 0);
                        if (U) {
                            const int pos = base + __popcll(want & ((1ull << lane) - 1ull));
                            // .y: the tile still holds an asymmetric cell (phase B then loads the regular mask)
                            Q[pos] = make_int4(t, (U & ~rg) ? 1 : 0, (int)(unsigned)(U & 0xFFFFFFFFull),
                                               (int)(unsigned)(U >> 32));
                        }
                    }
                }
                sync_global();
                if (tid == 0) { const unsigned long long n = __builtin_amdgcn_s_memtime(); ST(9, n - tmark); tmark = n; }
                const int qn = uni(S.qn);
                // ---- B: a wave per queued tile, lane = cell of the tile.  The tile-to-tile rows
                // (ttvis: a frontier tile every regular cell of t sees completely resolves them all;
                // ttany: no frontier tile in view of any regular cell of t, none is at this level)
                // and the cells' first runs (scan start, run count, hint, 4 heads -- coalesced, tile
                // order) are loaded in one round, independently of each other; the cells the rows
                // leave open then test the hint run, the heads and the next bext runs of their scan
                // order.  Misses go to the hard list.
                for (;;) {
                    // dynamic: the few tiles that need cell tests cost ~100x a row-resolved one; the regular
                    // mask is loaded only for tiles that hold an asymmetric cell (flagged in the entry), so
                    // the cell loads follow the entry without a round trip of their own
                    int it = 0;
                    if (lane == 0) it = atomicAdd(&S.bn, 1);
                    it = __builtin_amdgcn_readlane(it, 0);
                    if (it >= qn) break;
                    const int4 e = Q[it];
                    const int t = e.x;
                    unsigned long long mask = (unsigned long long)(unsigned)e.z | ((unsigned long long)(unsigned)e.w << 32);
                    const int id = (t << 6) | lane;
                    const unsigned long long reg = (SPECIAL && e.y) ? P.regular_tiles[t] : ~0ull;
                    const bool lreg = !SPECIAL || ((reg >> lane) & 1ull);
                    const bool cand = ((mask >> lane) & 1ull) && lreg;
                    int64_t ss = 0;
                    int nr = 0;
                    uint32_t hp = 0xFFFFFFFFu, hp2[VGA_H2];
#pragma unroll
                    for (int k = 0; k < VGA_H2; k++) hp2[k] = 0xFFFFFFFFu;
                    unsigned long long hmw = 0ull;   // (wide grids) a mask hint
                    int64_t pof = 0;
                    // heads loaded with the cell's first loads, the rest of the KH heads in the extension loop
                    // (round 4 at 1000^2: 4 -> 2 heads 4.67 -> 4.60 s, fewer live registers at the head tests)
                    constexpr int KH0 = 2;
                    unsigned long long hd0 = 0ull, hd1 = 0ull;
                    if (cand) {
                        ss = P.tscan_start[id];
                        nr = P.tnruns[id];
                        hp = Hn[id];
                        if (!FG && P.hint2)
#pragma unroll
                            for (int k = 0; k < VGA_H2; k++) hp2[k] = P.hint2[(size_t)k * nt * 64 + id];
                        if (FG && P.hintw) hmw = P.hintw[id];
                        if (P.pmask) pof = P.poff[id];
                        hd0 = run_word(P.heads + id);
                        hd1 = run_word(P.heads + hstride + id);
                    }
                    unsigned long long acc = 0ull, acca = ~0ull;
                    if (P.ttvis) {
                        acca = 0ull;
                        if (!FG) {   // (the host drops ttvis for a wide grid whose frontier fits the LDS)
#pragma unroll
                            for (int k = 0; k < 4; k++) {
                                const int w = k * 64 + lane;
                                const unsigned long long fs = w < P.tvw ? Fsr[w] : 0ull;
                                if (fs) {
                                    acc |= P.ttvis[(size_t)t * P.tvw + w] & fs;
                                    acca |= P.ttany[(size_t)t * P.tvw + w] & fs;
                                }
                            }
                        } else {
                            // wide rows (above 1024 cells a side): the words under frontier tile rows, 64 a round
#pragma unroll 1
                            for (int w = lane; w < P.tvw; w += 64) {
                                const unsigned long long fs = Fsr[w];
                                if (fs) {
                                    acc |= P.ttvis[(size_t)t * P.tvw + w] & fs;
                                    acca |= P.ttany[(size_t)t * P.tvw + w] & fs;
                                }
                            }
                        }
                    }
                    if (lane == 0) { ST(18, 1); ST(19, __popcll(mask)); }
                    if (__ballot(acc != 0ull) != 0ull) {
                        // a frontier tile every regular cell of t sees completely
                        const unsigned long long R = mask & reg;
                        if (lane == 0) { or_wg(&Xg[t], R); ST(20, 1); }
                        mask &= ~R;
                    } else if (__ballot(acca != 0ull) == 0ull) {
                        // no regular cell of t sees any frontier tile: none is at the next level
                        if (lane == 0) ST(25, 1);
                        mask &= ~reg;
                    }
                    const bool mine = (mask >> lane) & 1ull;
                    if (__ballot(mine) && lane == 0) ST(27, 1);
                    bool hit = false, to_hard = false;
                    int hard_val = 0;
                    if (mine && !lreg) {
                        to_hard = true;
                        hard_val = -1 - id;   // special node: exact path
                    } else if (mine) {
                        // The hint's operand (a run of the scan order, or a partial tile's mask) is loaded
                        // first and tested after the 4 heads, so the load overlaps the heads' LDS tests;
                        // a head hit leaves the hint alone (heads are tested every time anyway).
                        Run hr;
                        hr.x0 = -1;
                        unsigned long long hmk = 0ull;
                        int htile = -1;
                        if (FG && hmw && P.pmask) {
                            htile = (int)(hmw >> 32) - 1;
                            hmk = P.pmask[pof + (uint32_t)hmw];
                        } else if (hp != 0xFFFFFFFFu && (hp >> 31)) {
                            if (P.pmask) {   // a partial tile and its mask, or (slot 0xFFFF) a tile seen completely
                                htile = (int)((hp >> 16) & 0x7FFFu);
                                hmk = (hp & 0xFFFFu) == 0xFFFFu ? ~0ull : P.pmask[pof + (hp & 0xFFFFu)];
                            }
                        } else if (hp >= KH && hp < (uint32_t)nr) {
                            hr = P.scan_pool[ss + hp];
                        }
#pragma unroll 1
                        for (int r = 0; r < KH0; r++)
                            if (!hit && r < nr) {
                                rt++;
                                hit = run_hits_fs(FV, run_of(r == 0 ? hd0 : hd1));
                            }
                        if (!hit && htile >= 0) { rt++; hit = (F[htile] & hmk) != 0ull; }
                        else if (!hit && hr.x0 >= 0) { rt++; hit = run_hits_fs(FV, hr); }
#pragma unroll
                        for (int k = 0; k < VGA_H2; k++)   // fully seen tiles
                            if (!hit && hp2[k] != 0xFFFFFFFFu) { rt++; hit = F[(hp2[k] >> 16) & 0x7FFFu] != 0ull; }
                        // past the heads only in scan order: after the masks took the scan order's place (wide grids)
                        // the runs are in pool order, where positions KH.. are not the runs after the heads
                        const int next = (P.scan_pool == P.pool) ? KH : KH + P.bext;
                        const int lim = min(nr, next);
                        if (!hit) ST(29, 1);
                        bool skipped = false;
                        for (int base = KH0; base < lim && !hit; base += 4) {
                            Run rr[4];
#pragma unroll
                            for (int j = 0; j < 4; j++) {
                                const int r = base + j;
                                if (r < KH) rr[j] = P.heads[r * hstride + id];
                                else if (r < lim) rr[j] = P.scan_pool[ss + r];
                                else rr[j].x0 = -1;
                            }
                            // diagonal runs are left to phase C's exact mask test (their test walks the tiles)
                            if (P.pmask)
#pragma unroll
                                for (int j = 0; j < 4; j++)
                                    if (rr[j].x0 >= 0 && rr[j].x0 != rr[j].x1 && rr[j].y0 != rr[j].y1) {
                                        rr[j].x0 = -1;
                                        skipped = true;   // not a full test: a miss goes to phase C
                                    }
                            bool h4[4];
#pragma unroll
                            for (int j = 0; j < 4; j++) h4[j] = rr[j].x0 >= 0 && run_hits_fs(FV, rr[j]);
                            int fj = -1;
#pragma unroll
                            for (int j = 3; j >= 0; j--)
                                if (h4[j]) fj = j;
                            rt += (unsigned)min(4, lim - base);
                            if (fj >= 0) { hit = true; if (hp != (uint32_t)(base + fj)) Hn[id] = (uint32_t)(base + fj); }
                        }
                        if (!hit) {
                            if (nr > next || skipped) { to_hard = true; hard_val = id; }
                            else { ST(5, 1); ST(6, nr); }
                        }
                    }
                    const unsigned long long hm = __ballot(hit);
                    if (hm && lane == 0) or_wg(&Xg[t], hm);
                    const unsigned long long hw = __ballot(to_hard);
                    if (hw) {
                        int base = 0;
                        if (lane == 0) base = atomicAdd(&S.hn, __popcll(hw));
                        base = __shfl(base, 0);
                        if (to_hard) L[base + __popcll(hw & ((1ull << lane) - 1ull))] = hard_val;
                    }
                }
                sync_global();
                if (tid == 0) { const unsigned long long n = __builtin_amdgcn_s_memtime(); ST(10, n - tmark); tmark = n; }
                const int hn = uni(S.hn);
                // ---- C: hard cells.  A wave grabs CCH list entries at once (one coalesced load);
                // C0 tests their tile-visibility rows two cells at a time (16 row words a lane in
                // flight): a frontier tile the cell sees completely is a certain hit (regular cell:
                // in-set == out-set), no tile in view holding a frontier cell a certain miss.  C1
                // scans the run lists of the undecided cells, CSTEP * 64 runs a step (CSTEP loads a lane).
                constexpr int CCH = VGA_CCH;
                // runs a lane loads per scan step (1000^2: 4 -> 9.61 s, 8 -> 9.71 s, 16 -> 14.6 s: more loads
                // in flight per round trip do not pay for the registers and the over-read past the first hit)
                constexpr int CSTEP = 4;
                const unsigned long long c_t0 = __builtin_amdgcn_s_memtime();
                for (;;) {
                    int it0 = 0;
                    if (lane == 0) it0 = atomicAdd(&S.item, CCH);
                    it0 = __builtin_amdgcn_readlane(it0, 0);
                    if (it0 >= hn) break;
                    const int cn = min(CCH, hn - it0);
                    const int myv = lane < cn ? L[it0 + lane] : -1;
                    // the chunk's non-zero row summaries (tvnz), one load: lane 4j + k holds word k of entry j
                    static_assert(CCH * 4 <= 64, "tvnz prefetch: 4 summary words an entry");
                    unsigned long long nzp = ~0ull;
                    if (VGA_TVNZ && !FG && P.tvnz) {
                        const int jj = lane >> 2, kk = lane & 3, tvsw = (P.tvw + 63) >> 6;
                        const int vj = __shfl(myv, jj);
                        if (jj < cn && kk < tvsw) nzp = P.tvnz[(size_t)(vj < 0 ? -1 - vj : vj) * tvsw + kk];
                    }
                    unsigned long long certain_m = 0ull, pruned_m = 0ull;   // bit j: chunk entry j
                    if (P.tvis && (!P.pmask || (FG && VGA_WIDE_ROWPASS && P.tvsum))) {   // (wide grids: a row pass in front of the masks)
                        for (int j = 0; j < cn; j += 2) {
                            const int v0 = __builtin_amdgcn_readlane(myv, j);
                            const int v1 = __builtin_amdgcn_readlane(myv, j + 1);
                            const bool r0 = v0 >= 0, r1 = j + 1 < cn && v1 >= 0;
                            const unsigned long long* tv0 = P.tvis + (size_t)(r0 ? v0 : 0) * P.tvw;
                            const unsigned long long* tv1 = P.tvis + (size_t)(r1 ? v1 : 0) * P.tvw;
                            const unsigned long long* fv0 = P.ftvis ? P.ftvis + (size_t)(r0 ? v0 : 0) * P.tvw : nullptr;
                            const unsigned long long* fv1 = P.ftvis ? P.ftvis + (size_t)(r1 ? v1 : 0) * P.tvw : nullptr;
                            unsigned long long fa0 = 0ull, ta0 = 0ull, fa1 = 0ull, ta1 = 0ull;
                            if (!P.tvsum) {
                                // 4 row words a lane up to 1024 cells a side
#pragma unroll 4
                                for (int k = 0; k * 64 < P.tvw; k++) {
                                    const int w = k * 64 + lane;
                                    const unsigned long long fs = w < P.tvw ? Fsr[w] : 0ull;
                                    if (fs) {   // rows are read only under frontier tile rows
                                        if (r0) {
                                            ta0 |= tv0[w] & fs;
                                            if (fv0) fa0 |= fv0[w] & fs;
                                        }
                                        if (r1) {
                                            ta1 |= tv1[w] & fs;
                                            if (fv1) fa1 |= fv1[w] & fs;
                                        }
                                    }
                                }
                            } else {
                                // wider grids: the row summaries leave out the words that are zero for the
                                // cell (ftvis lies inside tvis); summary word k (lane k) holds bit `lane` for row word w
                                const int tvsw = (P.tvw + 63) / 64;
                                unsigned long long sm0 = 0ull, sm1 = 0ull;
                                if (lane < tvsw) {
                                    sm0 = r0 ? P.tvsum[(size_t)v0 * tvsw + lane] : 0ull;
                                    sm1 = r1 ? P.tvsum[(size_t)v1 * tvsw + lane] : 0ull;
                                }
                                for (int k = 0; k < tvsw; k++) {
                                    const int w = k * 64 + lane;
                                    const unsigned long long s0 =
                                        (unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)sm0, k) |
                                        ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)(sm0 >> 32), k) << 32);
                                    const unsigned long long s1 =
                                        (unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)sm1, k) |
                                        ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)(sm1 >> 32), k) << 32);
                                    if (!((s0 | s1) >> lane & 1ull)) continue;
                                    const unsigned long long fs = Fsr[w];   // w < tvw: its summary bit is set
                                    if (fs) {
                                        if ((s0 >> lane) & 1ull) {
                                            ta0 |= tv0[w] & fs;
                                            if (fv0) fa0 |= fv0[w] & fs;
                                        }
                                        if ((s1 >> lane) & 1ull) {
                                            ta1 |= tv1[w] & fs;
                                            if (fv1) fa1 |= fv1[w] & fs;
                                        }
                                    }
                                }
                            }
                            if (r0) {
                                if (__ballot(fa0 != 0ull)) certain_m |= 1ull << j;
                                else if (!__ballot(ta0 != 0ull)) pruned_m |= 1ull << j;
                            }
                            if (r1) {
                                if (__ballot(fa1 != 0ull)) certain_m |= 2ull << j;
                                else if (!__ballot(ta1 != 0ull)) pruned_m |= 2ull << j;
                            }
                        }
                        const unsigned long long regm = __ballot(lane < cn && myv >= 0);
                        if (lane == 0) {
                            ST(14, __popcll(regm));
                            ST(16, __popcll(certain_m));
                            ST(1, __popcll(certain_m));
                            ST(13, __popcll(pruned_m));
                        }
                    }
                    unsigned long long found_m = certain_m;
                    for (int j = 0; j < cn; j++) {
                        if (((certain_m | pruned_m) >> j) & 1ull) continue;
                        int id = __builtin_amdgcn_readlane(myv, j);
                        const bool special = id < 0;
                        if (special) id = -1 - id;
                        bool found = false;
                        int nr = 0;
                        unsigned nzb = 0xFu;   // row words k*64 + lane (k < 4) that are non-zero for the cell
                        if (VGA_TVNZ && !FG && P.tvnz) {
                            nzb = 0u;
#pragma unroll
                            for (int k = 0; k < 4; k++) {
                                const unsigned long long sk =
                                    (unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)nzp, j * 4 + k) |
                                    ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)(nzp >> 32), j * 4 + k) << 32);
                                nzb |= (unsigned)((sk >> lane) & 1ull) << k;
                            }
                        }
                        if (SPECIAL && special) {
                            int x, y;
                            xy_of_tile_id(id, tw, x, y);
                            int nmiss = 1;
                            if (P.pmask) found = special_extra_hit(P, F, P.cell_node[x * rows + y], &nmiss);
                            if (!found && nmiss == 0) {
                                // no Missing cell in the frontier: in-set meets F iff cells(v) does (the masks)
                                unsigned nl = 0;
                                int how = 0;
                                found = (FG && P.tvsum) ? pmask_hit_wide(P, F, Fsr, id, nl) : pmask_hit_fused(P, F, Fsr, id, nl, Hn, how, nzb);
                            } else if (!found) {
                                found = special_hit(P, FV, id, x, y, &nr);
                                if (lane == 0) rt += (unsigned)nr;
                            }
                            if (lane == 0) ST(24, 1);
                        } else if (P.pmask) {
                            unsigned nl = 0;
                            int how = 0;
#if VGA_PHASEC_OFF
                            found = false;   // attribution build: phase C reads nothing (results differ)
#elif VGA_ROWSTAT
                            unsigned rsv[3] = {0u, 0u, 0u};
                            found = (FG && P.tvsum) ? pmask_hit_wide(P, F, Fsr, id, nl) : pmask_hit_fused(P, F, Fsr, id, nl, Hn, how, nzb, rsv);
                            if (lane == 0) { ST(22, rsv[0]); ST(26, rsv[1]); ST(28, rsv[2]); }
#else
                            found = (FG && P.tvsum) ? pmask_hit_wide(P, F, Fsr, id, nl) : pmask_hit_fused(P, F, Fsr, id, nl, Hn, how, nzb);
#endif
                            if (lane == 0) {
                                ST(14, 1);
                                if (how == 1) { ST(16, 1); }
                                if (how == 2) ST(13, 1);
                            }
                            nl += __shfl_xor(nl, 32); nl += __shfl_xor(nl, 16); nl += __shfl_xor(nl, 8);
                            nl += __shfl_xor(nl, 4); nl += __shfl_xor(nl, 2); nl += __shfl_xor(nl, 1);
                            if (lane == 0) {
                                ST(30, nl);
                                ST(31, 1);
                                if (found) ST(1, 1);
                            }
                        } else {
                            const int64_t rs = P.tscan_start[id];
                            nr = P.tnruns[id];
                            // the first KH + bext runs were tested in phase B (in pool order -- the scan order
                            // released for the masks -- the heads are not the first runs: scan them all)
                            int base = P.scan_pool == P.pool ? 0 : KH + P.bext;
                            for (; base < nr && !found; base += CSTEP * 64) {
                                Run rr[CSTEP];
#pragma unroll
                                for (int k = 0; k < CSTEP; k++) {
                                    const int r = base + k * 64 + lane;
                                    if (r < nr) rr[k] = P.scan_pool[rs + r];
                                    else rr[k].x0 = -1;
                                }
                                // the tests are independent (no early-out between them), so their LDS
                                // round trips overlap
                                bool hk[CSTEP];
#pragma unroll
                                for (int k = 0; k < CSTEP; k++) hk[k] = rr[k].x0 >= 0 && run_hits_fs(FV, rr[k]);
                                int fpos = -1;
#pragma unroll
                                for (int k = CSTEP - 1; k >= 0; k--) {
                                    const unsigned long long hmk = __ballot(hk[k]);
                                    if (hmk) fpos = base + k * 64 + __ffsll((long long)hmk) - 1;
                                }
                                found = fpos >= 0;
                                if (found && lane == 0) Hn[id] = (uint32_t)fpos;
                            }
                            if (lane == 0) {
                                const unsigned long long sc = (unsigned long long)max(min(base, nr) - KH - P.bext, 0);
                                rt += (unsigned)sc;
                                ST(15, sc);
                                if (found) ST(1, 1);
                            }
                        }
                        if (found) found_m |= 1ull << j;
                        else if (lane == 0) ST(6, nr);
                    }
                    // publish the hits of the chunk (tile order: one atomic per entry that hit)
                    if (lane < cn && ((found_m >> lane) & 1ull)) {
                        const int id = myv < 0 ? -1 - myv : myv;
                        or_wg(&Xg[id >> 6], 1ull << (id & 63));
                    }
                    if (lane == 0) ST(5, cn - __popcll(found_m));
                }
                if (lane == 0) ST(21, __builtin_amdgcn_s_memtime() - c_t0);
            } else {
                // ---- top-down from the frontier F (small frontier): list it, then reuse F's LDS as
                // the bitmap the frontier's runs are pushed into
                for (int t = tid; t < nt; t += NT) {
                    unsigned long long f = F[t];
                    const int c = __popcll(f);
                    int pos = c ? atomicAdd(&S.hn, c) : 0;
                    while (f) {
                        const int b = __ffsll((long long)f) - 1;
                        f &= f - 1;
                        L[pos++] = (t << 6) | b;
                    }
                }
                sync_global();
                for (int t = tid; t < nt; t += NT) F[t] = 0ull;
                sync_global();
                const int fn = uni(S.hn);
                for (;;) {
                    int it = 0;
                    if (lane == 0) it = atomicAdd(&S.item, 1);
                    it = __builtin_amdgcn_readlane(it, 0);
                    if (it >= fn) break;
                    int x, y;
                    xy_of_tile_id(L[it], tw, x, y);
                    const int node = P.cell_node[x * rows + y];
                    const int64_t rs = P.node_run_start[node];
                    const int nr = P.node_nruns[node];
                    for (int r = lane; r < nr; r += 64) run_or(F, tw, P.pool[rs + r]);
                    if (lane == 0) rt += (unsigned)nr;
                }
                sync_global();
                for (int t = tid; t < nt; t += NT) Xg[t] = F[t] & ~Vg[t];
            }
            sync_global();
            if (P.asym_tiles) {
                // asymmetric mode: the frontier's A cells (listed by the last bookkeeping) push the graph's own runs
                // (a wave a cell, lanes over its runs) into F -- free until the bookkeeping rebuilds it, and in LDS
                // below 1024 cells a side -- and the unvisited part joins X
                const int an = min(uni(S.an), P.alist_cap);
                if (an > 0) {
                    unsigned long long* PB = F;
                    for (int t = tid; t < nt; t += NT) PB[t] = 0ull;
                    sync_global();
                    for (;;) {
                        int it = 0;
                        if (lane == 0) it = atomicAdd(&S.aitem, 1);
                        it = __builtin_amdgcn_readlane(it, 0);
                        if (it >= an) break;
                        int x, y;
                        xy_of_tile_id(P.alist[(size_t)blockIdx.x * P.alist_cap + it], tw, x, y);
                        const int an_node = P.cell_node[x * rows + y];
                        const int64_t rs = P.arun_start[an_node];
                        const int nr = P.anruns[an_node];
                        // 4 run loads in flight a lane (the loop is load-latency bound)
                        for (int r0 = 0; r0 < nr; r0 += 4 * 64) {
                            Run rr[4];
#pragma unroll
                            for (int k = 0; k < 4; k++) {
                                const int r = r0 + k * 64 + lane;
                                if (r < nr) rr[k] = P.apool[rs + r];
                                else rr[k].x0 = -1;
                            }
#pragma unroll
                            for (int k = 0; k < 4; k++)
                                if (rr[k].x0 >= 0) run_or(PB, tw, rr[k]);
                        }
                        if (lane == 0) rt += (unsigned)nr;
                    }
                    sync_global();
                    for (int t = tid; t < nt; t += NT) {
                        const unsigned long long pb = FG ? ld_wg(&PB[t]) : PB[t];
                        if (pb) {
                            const unsigned long long nw = pb & ~Vg[t];
                            if (nw) or_wg(&Xg[t], nw);
                        }
                    }
                }
                __syncthreads();
                if (tid == 0) { S.an = 0; S.aitem = 0; }
                __syncthreads();   // (before the bookkeeping appends the next level's A cells)
            }
            {
                const unsigned long long n = __builtin_amdgcn_s_memtime();
                if (tid == 0) {
                    if (bottom_up) ST(11, n - tmark);
                    else ST(level == 0 ? 8 : 17, n - tmark);
                }
                tmark = n;
            }
            // ---- level bookkeeping: count X, publish the expandable part as the next frontier
            // Walk the tiles listed for this level (all tiles after level 0: no list yet) -- X only ever
            // holds cells that were unvisited, so every other tile has none -- and list the tiles that
            // keep an unvisited cell for the next level.  A cleared frontier first: unlisted tiles
            // publish nothing (the merge pass may have set bits anywhere).
            const bool have_list = level > 0;
            for (int i = tid; i < nfs; i += NT) Fsr[i] = 0ull;
            if (have_list)
                for (int t = tid; t < nt; t += NT) F[t] = 0ull;
            __syncthreads();
            unsigned long long c_loc = 0, m_loc = 0;
            const int32_t* TLc = TL + (level & 1) * nt;
            int32_t* TLn = TL + ((level + 1) & 1) * nt;
            const int nwalk = have_list ? uni(S.tn[level & 1]) : nt;
            for (int i0 = 0; i0 < nwalk; i0 += NT) {
                const int t = i0 + tid < nwalk ? (have_list ? TLc[i0 + tid] : i0 + tid) : -1;
                bool open = false;
                if (t >= 0) {
                unsigned long long x = ld_wg(&Xg[t]);
                const unsigned long long v0 = Vg[t];
                open = ~(v0 | x) != 0ull;
                if (x) {
                    c_loc += (unsigned long long)__popcll(x);
                    Vg[t] = v0 | x;
                    Xg[t] = 0ull;
                    if (P.cell_level)
                        for (unsigned long long m = x; m; m &= m - 1) P.cell_level[t * 64 + __ffsll((long long)m) - 1] = level + 1;
                    // VGA global expands every cell when radius == n (vgavisualglobal.cpp:98-104);
                    // step depth never expands contextfilled odd cells (vgavisualglobaldepth.cpp:53)
                    if (P.radius != -1 || seeded) x &= ~P.nonexp_tiles[t];
                    m_loc += (unsigned long long)__popcll(x);
                    if (P.asym_tiles) {   // asymmetric mode: the A cells expand by pushing their own runs
                        unsigned long long xa = x & P.asym_tiles[t];
                        if (xa) {
                            x &= ~xa;
                            int pos = atomicAdd(&S.an, __popcll(xa));
                            int32_t* AL = P.alist + (size_t)blockIdx.x * P.alist_cap;
                            for (; xa; xa &= xa - 1)
                                if (pos < P.alist_cap) AL[pos++] = (t << 6) | (__ffsll((long long)xa) - 1);
                        }
                    }
                    if (x) {
                        const int tx = t % tw, ty = t / tw;
                        atomicOr(&Fsr[ty * wr + (tx >> 6)], 1ull << (tx & 63));
                        if (!RBM) atomicOr(&Fsc[tx * wc + (ty >> 6)], 1ull << (ty & 63));
                    }
                }
                F[t] = x;
                }
                const unsigned long long om = __ballot(open);
                if (om) {
                    int base = 0;
                    if (lane == 0) base = atomicAdd(&S.tn[(level + 1) & 1], __popcll(om));
                    base = __shfl(base, 0);
                    if (open) TLn[base + __popcll(om & ((1ull << lane) - 1ull))] = t;
                }
            }
            for (int off = 32; off >= 1; off >>= 1) {
                c_loc += __shfl_xor(c_loc, off);
                m_loc += __shfl_xor(m_loc, off);
            }
            if (lane == 0 && c_loc) { atomicAdd(&S.cnt, c_loc); atomicAdd(&S.mass, m_loc); }
            if (P.nmp && (P.radius == -1 || level + 1 < P.radius)) {
                __syncthreads();   // the new level is in F and V
                merge_level_pass(P.mpairs, P.nmp, rows, tw, NT, F, Vg, false, P.seed_tiles, Fsr, RBM ? nullptr : Fsc, wr,
                                 wc, P.cell_level, level + 1, &S.mcorr, &S.mdisc, &S.mass);
                if (P.nmamb && !seeded) {
                    __syncthreads();
                    merge_order_check(P.mamb, P.nmamb, rows, tw, NT, F, Vg, false, P.seed_tiles,
                                      P.mseen + (size_t)blockIdx.x * P.nmamb, (int32_t)node + 1, P.error, P.oflag, node);
                }
            }
            if (RBM) {
                // line-resolved summaries from the published frontier (plain stores, no atomics)
                __syncthreads();
                const int th = P.th;
                // one thread per (tile row, word) builds that word's 8 row summaries from the frontier tiles
                // Fsr lists, one per (tile column, word) its 8 column summaries: each F word read once
                for (int i = tid; i < th * wr + tw * wc; i += NT) {
                    unsigned long long b[8];
#pragma unroll
                    for (int k = 0; k < 8; k++) b[k] = 0ull;
                    if (i < th * wr) {
                        const int ty = i / wr, w = i % wr;
                        const unsigned long long* fr = F + ty * tw + w * 64;
                        for (unsigned long long m = Fsr[ty * wr + w]; m; m &= m - 1) {
                            const int j = __ffsll((long long)m) - 1;
                            const unsigned long long f = fr[j];
#pragma unroll
                            for (int k = 0; k < 8; k++) b[k] |= (unsigned long long)(((f >> (8 * k)) & 0xFFull) != 0ull) << j;
                        }
#pragma unroll
                        for (int k = 0; k < 8; k++) RB[(ty * 8 + k) * wr + w] = b[k];
                    } else {
                        const int q = i - th * wr, tx = q / wc, w = q % wc;
                        const int n = min(64, th - w * 64);
                        for (int j = 0; j < n; j++) {
                            unsigned long long y = F[(w * 64 + j) * tw + tx];
                            y |= y >> 32;
                            y |= y >> 16;
                            y |= y >> 8;
#pragma unroll
                            for (int k = 0; k < 8; k++) b[k] |= ((y >> k) & 1ull) << j;
                        }
#pragma unroll
                        for (int k = 0; k < 8; k++) CB[(tx * 8 + k) * wc + w] = b[k];
                    }
                }
            }
            sync_global();
            const long long cnt = uni64(S.cnt), mass = uni64(S.mass);
            const long long mcorr = uni64(S.mcorr), mdisc = uni64(S.mdisc);
            if (tid == 0) { const unsigned long long n = __builtin_amdgcn_s_memtime(); ST(12, n - tmark); tmark = n; }
            __syncthreads();
            if (tid == 0) {
                S.cnt = 0; S.mass = 0; S.qn = 0; S.hn = 0; S.item = 0; S.bn = 0; S.mcorr = 0; S.mdisc = 0;
                S.tn[level & 1] = 0;   // this level's list is spent; it is the next level's append target
                S.disc += cnt + mdisc;
                S.m_u -= cnt + mdisc;
                S.m_f = mass;
            }
            // the next level's first appends (phase A's queue, the top-down frontier list) must not race
            // the resets above: a wave that appended before them lost its entries
            __syncthreads();
            if (cnt == 0) break;
            if (level + 1 >= VGA_HMAX) { overflow = true; break; }
            if (tid == 0) hist[level + 1] = (int)(cnt - mcorr);
            level++;
            nlev = level + 1;
            if (tid == 0) ST(bottom_up ? 3 : 4, 1);
        }
        __syncthreads();
        if (overflow) {
            // the source's histogram is incomplete: marked skipped (0 levels) so that the measures kernel, launched
            // before the host reads the error and falls back to vga_do, reads none of it (it used to read this
            // source's unwritten level count)
            if (tid == 0) { atomicOr(P.error, KERR_LEVELS); P.nlev_out[node] = 0; }
            continue;
        }
        {   // flush this lane-group's run-test count (32-bit per lane, per source)
            unsigned r = rt;
            for (int off = 32; off >= 1; off >>= 1) r += __shfl_xor(r, off);
            if (lane == 0 && r) ST(0, r);
            rt = 0;
        }
        for (int l = tid; l < nlev; l += NT) P.hist_out[node * VGA_HMAX + l] = hist[l];
        if (tid == 0) P.nlev_out[node] = nlev;
        __syncthreads();
    }
    for (int off = 32; off >= 1; off >>= 1) rt += __shfl_xor(rt, off);
    if (lane == 0 && rt) ST(0, rt);
    __syncthreads();
    for (int i = tid; i < 32; i += NT)
        if (SC[i]) atomicAdd(&P.stats[i], SC[i]);
#undef ST
}

// ---------------------------------------------------------------- prep: tile-ordered cell arrays
__device__ __forceinline__ int run_len(Run ru) {
    return max(ru.x1 - ru.x0, max(ru.y1 - ru.y0, ru.y0 - ru.y1)) + 1;
}

// Tile-ordered scan start / run count per cell, and its KH head runs (the first KH entries of its
// scan order: the longest run of each angular group).  One thread per node.
__global__ void tile_heads_kernel(int rows, int tw, const int32_t* node_cell, int64_t n, const int32_t* node_nruns,
                                  const Run* scan_pool, const int64_t* scan_start, int64_t* tscan_start, int32_t* tnruns,
                                  Run* heads, size_t hstride) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const int c = node_cell[k];
    const int id = tile_id_of(c / rows, c % rows, tw);
    const int64_t ss = scan_start[k];
    const int nr = node_nruns[k];
    tscan_start[id] = ss;
    tnruns[id] = nr;
    // the first KH scan entries with the row / column runs before the diagonal ones (a diagonal run's
    // test walks its tiles one LDS round trip per 8; a row or column run costs <= 4 reads): the order
    // only changes which test hits first
    int o = 0;
    for (int pass = 0; pass < 2; pass++)
        for (int h = 0; h < KH && h < nr; h++) {
            const Run ru = scan_pool[ss + h];
            const bool diag = ru.x0 != ru.x1 && ru.y0 != ru.y1;
            if (diag == (pass == 1)) heads[(o++) * hstride + id] = ru;
        }
}

// Tile-visibility rows: bit (ty, tx) of cell id's row is set iff the cell sees some cell of tile
// (tx, ty); same [th][ceil(tw/64)] word layout as the kernel's Fsr summary, so one AND per word
// tells whether any frontier tile is in view.  The full-visibility row (ftvis) sets the bit only
// when the cell sees EVERY discoverable (non-seed) cell of the tile: a frontier tile under such a
// bit is a certain hit for a regular cell (in-set == out-set), so phase C resolves it without a run
// scan.  One workgroup (TV_WAVES waves, threads over the runs) per node; the rows and the per-tile
// covered-cell counts (bytes) are built in LDS with atomics.  A node per workgroup rather than per
// wave keeps the LDS per CU small enough for 4 workgroups (32 waves): the run walks are latency
// bound (divergent per-tile LDS atomics), so occupancy is what pays (1000^2: 0.33 s at 4 waves/CU).
constexpr int TV_WAVES = 8;
__device__ __forceinline__ void tv_count(uint32_t* cnt, int t, int c) {
    atomicAdd(&cnt[t >> 2], (uint32_t)c << (8 * (t & 3)));
}
__global__ void __launch_bounds__(64 * TV_WAVES) tile_vis_kernel(int rows, int tw, int th, const int32_t* node_cell,
                                                                 int64_t n, const int64_t* node_run_start,
                                                                 const int32_t* node_nruns, const Run* pool,
                                                                 const unsigned long long* seed_tiles,
                                                                 unsigned long long* tvis, unsigned long long* ftvis) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long tvlds[];
    const int nt = tw * th, ncw = (nt + 3) / 4;
    const int wr = (tw + 63) / 64, tvw = th * wr;
    constexpr int TB = 64 * TV_WAVES;
    const int tid = threadIdx.x;
    uint8_t* nsc = (uint8_t*)tvlds;                                   // [nt] non-seed cells per tile
    unsigned long long* row = tvlds + (ncw + 1) / 2;                  // [tvw]
    uint32_t* cnt = (uint32_t*)(row + tvw);                            // [nt] covered non-seed cells (bytes)
    if (ftvis)
        for (int t = tid; t < nt; t += TB) nsc[t] = (uint8_t)__popcll(~seed_tiles[t]);
    for (int64_t k = blockIdx.x; k < n; k += gridDim.x) {
        __syncthreads();   // the previous node's rows are written out
        for (int w = tid; w < tvw; w += TB) row[w] = 0ull;
        if (ftvis)
            for (int w = tid; w < ncw; w += TB) cnt[w] = 0u;
        __syncthreads();
        const int64_t rs = node_run_start[k];
        const int nr = node_nruns[k];
        for (int r = tid; r < nr; r += TB) {
            const Run ru = pool[rs + r];
            if (ru.y0 == ru.y1) {
                const int y = ru.y0, ty = y >> 3, t0 = ru.x0 >> 3, t1 = ru.x1 >> 3;
                for (int w = t0 >> 6; w <= (t1 >> 6); w++) {
                    const int lo = max(t0 - w * 64, 0), hi = min(t1 - w * 64, 63);
                    atomicOr(&row[ty * wr + w], (~0ull << lo) & (~0ull >> (63 - hi)));
                }
                if (ftvis)
                    for (int tx = t0; tx <= t1; tx++) {
                        const int a = max((int)ru.x0, tx * 8) & 7, b = min((int)ru.x1, tx * 8 + 7) & 7;
                        const unsigned long long m = (unsigned long long)((0xFFu >> (7 - b)) & (0xFFu << a) & 0xFFu) << ((y & 7) * 8);
                        const int t = ty * tw + tx;
                        const int c = __popcll(m & ~seed_tiles[t]);
                        if (c) tv_count(cnt, t, c);
                    }
            } else if (ru.x0 == ru.x1) {
                const int x = ru.x0, tx = x >> 3;
                const unsigned long long colm = 0x0101010101010101ull << (x & 7);
                for (int ty = ru.y0 >> 3; ty <= (ru.y1 >> 3); ty++) {
                    atomicOr(&row[ty * wr + (tx >> 6)], 1ull << (tx & 63));
                    if (ftvis) {
                        const int a = max((int)ru.y0, ty * 8) & 7, b = min((int)ru.y1, ty * 8 + 7) & 7;
                        const unsigned long long m = colm & (~0ull >> (8 * (7 - b))) & (~0ull << (8 * a));
                        const int t = ty * tw + tx;
                        const int c = __popcll(m & ~seed_tiles[t]);
                        if (c) tv_count(cnt, t, c);
                    }
                }
            } else {
                const int dy = (ru.y1 > ru.y0) ? 1 : -1;
                int x = ru.x0, y = ru.y0;
                while (x <= ru.x1) {
                    int n;
                    const unsigned long long m = diag_tile_mask(x, y, dy, ru.x1, n);
                    const int tx = x >> 3, ty = y >> 3;
                    atomicOr(&row[ty * wr + (tx >> 6)], 1ull << (tx & 63));
                    if (ftvis) {
                        const int t = ty * tw + tx;
                        const int c = __popcll(m & ~seed_tiles[t]);
                        if (c) tv_count(cnt, t, c);
                    }
                    x += n;
                    y += dy * n;
                }
            }
        }
        __syncthreads();
        const int c = node_cell[k];
        const int id = tile_id_of(c / rows, c % rows, tw);
        unsigned long long* out = tvis + (size_t)id * tvw;
        for (int w = tid; w < tvw; w += TB) out[w] = row[w];
        if (ftvis) {
            // a tile is fully seen when the covered count reaches its non-seed count (a node's runs
            // are disjoint, so no cell is counted twice)
            unsigned long long* fout = ftvis + (size_t)id * tvw;
            for (int w = tid; w < tvw; w += TB) {
                unsigned long long m = row[w], f = 0ull;
                const int tyw = w / wr, tx0 = (w % wr) * 64;
                while (m) {
                    const int j = __ffsll((long long)m) - 1;
                    m &= m - 1;
                    const int t = tyw * tw + tx0 + j;
                    const int cv = (cnt[t >> 2] >> (8 * (t & 3))) & 0xFF;
                    if (cv == nsc[t] && cv > 0) f |= 1ull << j;
                }
                fout[w] = f;
            }
        }
    }
}

// Partial tiles per cell: popcount of tvis & ~ftvis over its row, and the exclusive prefix of the
// per-word counts (ppre: the masks of word w start at ppre[w] within the cell's list).  One wave per
// cell, lane over words (tvw <= 256, so a cell has at most 16,384 partial tiles: u16).
__global__ void tile_pcount_kernel(int64_t Ct, int tvw, const unsigned long long* tvis, const unsigned long long* ftvis,
                                   int64_t* pcount, uint16_t* ppre) {
    const int lane = threadIdx.x & 63;
    const int64_t id = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (id >= Ct) return;
    int run = 0;
    for (int k = 0; k * 64 < tvw; k++) {
        const int w = k * 64 + lane;
        const int c = w < tvw ? __popcll(tvis[id * tvw + w] & ~ftvis[id * tvw + w]) : 0;
        const int incl = wave_incl_scan(c);
        if (w < tvw) ppre[id * tvw + w] = (uint16_t)(run + incl - c);
        run += __builtin_amdgcn_readlane(incl, 63);
    }
    if (lane == 0) pcount[id] = run;
}

// Partial-tile masks: for every tile a cell sees only in part (tvis & ~ftvis), the 64-bit mask of the
// tile's cells it sees, stored at pmask[poff[id] + rank] with rank = partial bits before the tile in
// row-word then bit order.  One workgroup per node walks the node's runs as tile_vis_kernel does and
// ORs the per-tile masks into LDS slots (global atomics for a node with more than pmcap partial
// tiles; pmask is zeroed beforehand).  A node's runs are disjoint, so every seen cell is one bit.
// Dynamic LDS: the partial words and their prefix [tvw] and the slots [pmcap] (tile_pmask_lds).
constexpr int PM_CAP = 4096;        // slots in LDS up to 1024 cells a side
constexpr int PM_CAP_WIDE = 8192;   // wider grids (a cell sees ~2,500 partial tiles at 2000^2)
__host__ __device__ inline size_t tile_pmask_lds(int tvw, int pmcap) { return (size_t)tvw * 12 + (size_t)pmcap * 8; }
__global__ void __launch_bounds__(64 * TV_WAVES) tile_pmask_kernel(int rows, int tw, int th, const int32_t* node_cell,
                                                                   int64_t n, const int64_t* node_run_start,
                                                                   const int32_t* node_nruns, const Run* pool,
                                                                   const unsigned long long* tvis,
                                                                   const unsigned long long* ftvis, const int64_t* poff,
                                                                   unsigned long long* pmask, int pmcap) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long pmlds[];
    __shared__ int ptotal;
    const int wr = (tw + 63) / 64, tvw = th * wr;
    unsigned long long* part = pmlds;             // [tvw]
    unsigned long long* lm = part + tvw;          // [pmcap]
    int* pre = (int*)(lm + pmcap);                // [tvw]
    constexpr int TB = 64 * TV_WAVES;
    const int tid = threadIdx.x, lane = tid & 63;
    for (int64_t k = blockIdx.x; k < n; k += gridDim.x) {
        const int c = node_cell[k];
        const int id = tile_id_of(c / rows, c % rows, tw);
        __syncthreads();   // the previous node's masks are written out
        if (tid < 64) {
            // partial words and their exclusive popcount prefix
            int run = 0;
            for (int kk = 0; kk * 64 < tvw; kk++) {
                const int w = kk * 64 + lane;
                const unsigned long long p = w < tvw ? (tvis[(size_t)id * tvw + w] & ~ftvis[(size_t)id * tvw + w]) : 0ull;
                const int cnt = __popcll(p);
                const int incl = wave_incl_scan(cnt);
                if (w < tvw) {
                    part[w] = p;
                    pre[w] = run + incl - cnt;
                }
                run += __builtin_amdgcn_readlane(incl, 63);
            }
            if (lane == 0) ptotal = run;
        }
        __syncthreads();
        const int P = ptotal;
        const bool in_lds = P <= pmcap;
        unsigned long long* gout = pmask + poff[id];
        if (in_lds)
            for (int i = tid; i < P; i += TB) lm[i] = 0ull;
        __syncthreads();
        auto put = [&](int tx, int ty, unsigned long long m) {
            const int w = ty * wr + (tx >> 6), b = tx & 63;
            const unsigned long long pwv = part[w];
            if (!((pwv >> b) & 1ull)) return;
            const int slot = pre[w] + __popcll(pwv & ((1ull << b) - 1ull));
            if (in_lds) atomicOr(&lm[slot], m);
            else atomicOr(&gout[slot], m);
        };
        const int64_t rs = node_run_start[k];
        const int nr = node_nruns[k];
        for (int r = tid; r < nr; r += TB) {
            const Run ru = pool[rs + r];
            if (ru.y0 == ru.y1) {
                const int y = ru.y0, ty = y >> 3;
                for (int tx = ru.x0 >> 3; tx <= (ru.x1 >> 3); tx++) {
                    const int a = max((int)ru.x0, tx * 8) & 7, b = min((int)ru.x1, tx * 8 + 7) & 7;
                    put(tx, ty, (unsigned long long)((0xFFu >> (7 - b)) & (0xFFu << a) & 0xFFu) << ((y & 7) * 8));
                }
            } else if (ru.x0 == ru.x1) {
                const int x = ru.x0, tx = x >> 3;
                const unsigned long long colm = 0x0101010101010101ull << (x & 7);
                for (int ty = ru.y0 >> 3; ty <= (ru.y1 >> 3); ty++) {
                    const int a = max((int)ru.y0, ty * 8) & 7, b = min((int)ru.y1, ty * 8 + 7) & 7;
                    put(tx, ty, colm & (~0ull >> (8 * (7 - b))) & (~0ull << (8 * a)));
                }
            } else {
                const int dy = (ru.y1 > ru.y0) ? 1 : -1;
                int x = ru.x0, y = ru.y0;
                while (x <= ru.x1) {
                    int nn;
                    const unsigned long long m = diag_tile_mask(x, y, dy, ru.x1, nn);
                    put(x >> 3, y >> 3, m);
                    x += nn;
                    y += dy * nn;
                }
            }
        }
        __syncthreads();
        if (in_lds)
            for (int i = tid; i < P; i += TB) gout[i] = lm[i];
    }
}

// Runs in pool order for the tile search (the scan order released for the wide-grid masks): each cell's
// first run is its node's first run in the pool.
__global__ void tile_pool_order_kernel(int rows, int tw, const int32_t* node_cell, int64_t n, const int64_t* node_run_start,
                                       int64_t* tscan_start) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const int c = node_cell[k];
    tscan_start[tile_id_of(c / rows, c % rows, tw)] = node_run_start[k];
}

// Tile-to-tile full visibility: row t = AND of the ftvis rows of tile t's regular cells (bit u set
// iff every regular cell of t sees every non-seed cell of tile u).  One wave per tile.
// ttany row t = OR of the tvis rows of t's regular cells (tiles some regular cell of t sees at all):
// no frontier tile under it means no regular cell of t can be reached at this level.
__global__ void tile_tt_kernel(int nt, int tvw, const unsigned long long* regular_tiles, const unsigned long long* ftvis,
                               const unsigned long long* tvis, unsigned long long* ttvis, unsigned long long* ttany) {
    const int lane = threadIdx.x & 63;
    const int t = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (t >= nt) return;
    const unsigned long long R = regular_tiles[t];
    for (int w = lane; w < tvw; w += 64) {
        unsigned long long acc = R ? ~0ull : 0ull, any = 0ull;
        for (unsigned long long m = R; m; m &= m - 1) {
            const int b = __ffsll((long long)m) - 1;
            acc &= ftvis[((size_t)t * 64 + b) * tvw + w];
            any |= tvis[((size_t)t * 64 + b) * tvw + w];
        }
        ttvis[(size_t)t * tvw + w] = acc;
        ttany[(size_t)t * tvw + w] = any;
    }
}

// Row summary of the tile-visibility rows (wide grids: tvsum; up to 256 words: tvnz): bit w of a cell's
// summary is set iff its row word w is non-zero, so phase C's miss certificate reads only the words the
// cell has (a dense map's cell sees a few % of the tiles) instead of every word under a frontier tile row.
// One wave per cell: summary word j is the ballot of row words 64j .. 64j + 63 being non-zero.
__global__ void tile_vsum_kernel(int64_t Ct, int tvw, const unsigned long long* tvis, unsigned long long* tvsum) {
    const int lane = threadIdx.x & 63;
    const int64_t c = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (c >= Ct) return;
    const int tvsw = (tvw + 63) / 64;
    const unsigned long long* row = tvis + (size_t)c * tvw;
    for (int j = 0; j < tvsw; j++) {
        const int w = j * 64 + lane;
        const unsigned long long bits = __ballot(w < tvw && row[w] != 0ull);
        if (lane == 0) tvsum[(size_t)c * tvsw + j] = bits;
    }
}

// Lattice segment: cells (x0 + p*dx, y0 + p*dy), p = 0..len-1 (dx in {0,1}, dy in {-1,0,1}).
struct LSeg {
    int x0, y0, dx, dy, len;
};
__device__ __forceinline__ LSeg lseg_of(Run ru) {
    LSeg s;
    s.x0 = ru.x0;
    s.y0 = ru.y0;
    if (ru.y0 == ru.y1) { s.dx = 1; s.dy = 0; s.len = ru.x1 - ru.x0 + 1; }
    else if (ru.x0 == ru.x1) { s.dx = 0; s.dy = 1; s.len = ru.y1 - ru.y0 + 1; }
    else { s.dx = 1; s.dy = (ru.y1 > ru.y0) ? 1 : -1; s.len = ru.x1 - ru.x0 + 1; }
    return s;
}
// Positions [*pa, *pb] of candidate `c` covered by segment `s` (empty if *pa > *pb).
__device__ __forceinline__ void lseg_overlap(const LSeg& c, const LSeg& s, int* pa, int* pb) {
    *pa = 1;
    *pb = 0;
    const int ux = s.x0 - c.x0, uy = s.y0 - c.y0;
    const int det = -c.dx * s.dy + s.dx * c.dy;
    if (det == 0) {
        // parallel: same lattice line iff (ux, uy) is collinear with (dx, dy)
        if (ux * c.dy - uy * c.dx != 0) return;
        const int a = c.dx ? ux : uy;
        *pa = max(a, 0);
        *pb = min(a + s.len - 1, c.len - 1);
        return;
    }
    // p*c.d - q*s.d = u  (Cramer)
    const int pn = -ux * s.dy + s.dx * uy, qn = c.dx * uy - c.dy * ux;
    if (pn % det != 0 || qn % det != 0) return;
    const int p = pn / det, q = qn / det;
    if (p < 0 || p >= c.len || q < 0 || q >= s.len) return;
    *pa = p;
    *pb = p;
}

// CR(t): up to two runs whose cells are visible from every regular cell of tile t.  Candidates are
// the group-longest runs of the tile's most central regular cell; every regular cell's runs are
// intersected with them through LDS difference arrays (O(runs) per tile).
constexpr int CR_THREADS = 256;
__global__ void __launch_bounds__(CR_THREADS) tile_cr_kernel(int cols, int rows, int tw, int th,
                                                             const unsigned long long* regular_tiles,
                                                             const int32_t* cell_node, const int64_t* node_run_start,
                                                             const int32_t* node_nruns, const int64_t* scan_start,
                                                             const Run* scan_pool, const Run* pool, int dmax, Run* cr) {
    extern __shared__ __attribute__((aligned(16))) int diff[];   // [8][dmax + 2]
    __shared__ LSeg cand[8];
    __shared__ int bestlen[8], beststart[8];
    const int nt = tw * th;
    const int tid = threadIdx.x;
    const int stride = dmax + 2;
    for (int t = blockIdx.x; t < nt; t += gridDim.x) {
        const unsigned long long R = regular_tiles[t];
        const int tx = t % tw, ty = t / tw;
        if (R == 0ull) {
            if (tid < CRK) { Run z; z.x0 = z.y0 = z.x1 = z.y1 = -1; cr[CRK * t + tid] = z; }
            continue;
        }
        const int nreg = __popcll(R);
        // most central regular cell (ties: lowest bit); its first 8 scan entries are the candidates
        int cb = 0, cd = 1 << 30;
        for (int b = 0; b < 64; b++)
            if ((R >> b) & 1ull) {
                const int d = (2 * (b & 7) - 7) * (2 * (b & 7) - 7) + (2 * (b >> 3) - 7) * (2 * (b >> 3) - 7);
                if (d < cd) { cd = d; cb = b; }
            }
        const int ck = cell_node[(tx * 8 + (cb & 7)) * rows + ty * 8 + (cb >> 3)];
        for (int i = tid; i < 8 * stride; i += CR_THREADS) diff[i] = 0;
        if (tid < 8) {
            const int nrc = node_nruns[ck];
            if (tid < nrc) cand[tid] = lseg_of(scan_pool[scan_start[ck] + tid]);
            else cand[tid].len = 0;
        }
        __syncthreads();
        // coverage counts: every regular cell's runs against the 8 candidates (difference arrays;
        // one cell's runs are disjoint, so a position counts each regular cell at most once)
        for (int b = 0; b < 64; b++) {
            if (!((R >> b) & 1ull)) continue;
            const int wk = cell_node[(tx * 8 + (b & 7)) * rows + ty * 8 + (b >> 3)];
            const int64_t rs = node_run_start[wk];
            const int nr = node_nruns[wk];
            for (int r = tid; r < nr; r += CR_THREADS) {
                const LSeg s = lseg_of(pool[rs + r]);
                for (int g = 0; g < 8; g++) {
                    const LSeg c = cand[g];
                    if (c.len == 0) continue;
                    int pa, pb;
                    lseg_overlap(c, s, &pa, &pb);
                    if (pa <= pb) {
                        atomicAdd(&diff[g * stride + pa], 1);
                        atomicAdd(&diff[g * stride + pb + 1], -1);
                    }
                }
            }
        }
        __syncthreads();
        if (tid < 8) {
            const LSeg c = cand[tid];
            int bl = 0, bs = 0, cur = 0, run = 0, rstart = 0;
            for (int p = 0; p < c.len; p++) {
                cur += diff[tid * stride + p];
                if (cur == nreg) {
                    if (run == 0) rstart = p;
                    run++;
                    if (run > bl) { bl = run; bs = rstart; }
                } else {
                    run = 0;
                }
            }
            bestlen[tid] = bl;
            beststart[tid] = bs;
        }
        __syncthreads();
        if (tid == 0) {
            // the CRK longest common intervals, longest first
            int used = 0;
            for (int j = 0; j < CRK; j++) {
                int pick = -1;
                // row / column runs first (cheap tests), longest first within each kind
                auto key = [&](int g) { return bestlen[g] + ((cand[g].dx == 0 || cand[g].dy == 0) ? (1 << 20) : 0); };
                for (int g = 0; g < 8; g++)
                    if (bestlen[g] > 0 && !((used >> g) & 1) && (pick < 0 || key(g) > key(pick))) pick = g;
                Run z;
                z.x0 = z.y0 = z.x1 = z.y1 = -1;
                if (pick >= 0) {
                    used |= 1 << pick;
                    const LSeg c = cand[pick];
                    const int pa = beststart[pick], pb = pa + bestlen[pick] - 1;
                    z.x0 = (int16_t)(c.x0 + pa * c.dx);
                    z.y0 = (int16_t)(c.y0 + pa * c.dy);
                    z.x1 = (int16_t)(c.x0 + pb * c.dx);
                    z.y1 = (int16_t)(c.y0 + pb * c.dy);
                }
                cr[CRK * t + j] = z;
            }
        }
        __syncthreads();
    }
}

// K4: the 7 VGA measures per source from its level histogram (vgavisualglobal.cpp:131-193).
// hist_all / nlev_all are indexed by source, or (by_index: vga_ordered's re-runs) by position in src_list, with
// hstride levels a row
// Asymmetric mode's A (dmx_api.hip prepare_asym): flag each node whose bins or runs differ between graphs a and b
// (same nodes).  One thread a node.
__global__ void node_runs_differ_kernel(int64_t n, const int32_t* bins_a, const int64_t* rs_a, const int32_t* nr_a,
                                        const Run* pool_a, const int32_t* bins_b, const int64_t* rs_b, const int32_t* nr_b,
                                        const Run* pool_b, uint8_t* out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    bool d = nr_a[k] != nr_b[k];
    for (int b = 0; b < 32 && !d; b++) d = bins_a[k * 32 + b] != bins_b[k * 32 + b];
    const unsigned long long* ra = (const unsigned long long*)(pool_a + rs_a[k]);
    const unsigned long long* rb = (const unsigned long long*)(pool_b + rs_b[k]);
    for (int r = 0; r < nr_a[k] && !d; r++) d = ra[r] != rb[r];
    out[k] = d ? 1 : 0;
}

__global__ void vga_measures_kernel(int64_t sb, int64_t se, const int32_t* hist_all, const int32_t* nlev_all, float* out,
                                    int64_t* levels_out, unsigned long long* stats, const int32_t* src_list = nullptr,
                                    int hstride = VGA_HMAX, bool by_index = false) {
    const int64_t i = sb + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= se) return;
    const int64_t src = src_list ? (int64_t)src_list[i] : i;
    const int64_t hi = by_index ? i : src;
    const int nlev = nlev_all[hi];
    float* o = out + src * 7;
    if (nlev <= 0 || nlev > hstride) {   // skipped source (context-filled odd cell / gates_only; a level overflow)
        for (int i = 0; i < 7; i++) o[i] = -1.0f;
        if (levels_out) { levels_out[src * 3] = 0; levels_out[src * 3 + 1] = 0; levels_out[src * 3 + 2] = 0; }
        return;
    }
    long long tn, td;
    vga_measures(hist_all + hi * hstride, nlev, o, tn, td);
    if (levels_out) {
        levels_out[src * 3 + 0] = tn;
        levels_out[src * 3 + 1] = td;
        levels_out[src * 3 + 2] = nlev;
    }
    atomicAdd(&stats[2], (unsigned long long)tn);
}

} // namespace dmx
