// common.hpp -- shared device-side definitions for the dmx HIP kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "../host/geometry.hpp"

namespace dmx {

constexpr int WAVE = 64;

// Kernel parameters read through a pointer to device memory (the persistent kernels: a large struct, its cold
// fields reloaded with scalar loads instead of held in SGPRs).  Read through the constant address space, so
// the compiler knows the pointers inside it are global: their loads, stores and atomics are global_* ops.
// Through a generic pointer they would be flat_* ops, which count against both the memory and the LDS
// counters and return out of order, so every use of a loaded value waits for all LDS and memory operations
// in flight (vmcnt(0) lgkmcnt(0)).
// (The host pass only type-checks the kernels; there the qualifier is left out.)
#if defined(__HIP_DEVICE_COMPILE__)
#define DMX_CONST_AS __attribute__((address_space(4)))
#else
#define DMX_CONST_AS
#endif
template <typename T>
__device__ __forceinline__ const DMX_CONST_AS T& const_params(const T* p) {
    return *(const DMX_CONST_AS T*)p;
}

// Error flags raised by kernels (bitwise OR into a device word; the host maps them to status codes).
enum KernelError : int {
    KERR_GAP_CAPACITY = 1,     // sieve gap list exceeded LDS capacity
    KERR_BLOCK_CAPACITY = 2,   // per-depth block list exceeded LDS capacity
    KERR_STAGE_CAPACITY = 4,   // per-source run staging exceeded scratch capacity
    KERR_POOL_CAPACITY = 8,    // global run pool exhausted
    KERR_BIN_MISMATCH = 16,    // whichbin produced a bin outside the octant (should never happen)
    KERR_LEVELS = 32,          // BFS depth exceeded the level histogram
    KERR_FRONTIER = 64,        // BFS frontier buffer overflow
    KERR_ORDER = 128,          // a merge-link outcome depends on the reference's pop order (merge_order_check)
};

// Per-cell word uploaded to HBM: bit 0 FILLED, bits 1..7 cropped-segment count (<=127),
// bits 8..31 offset of the cell's first segment.
__host__ __device__ inline uint32_t pack_cell(bool filled, uint32_t nseg, uint32_t off) {
    return (off << 8) | (nseg << 1) | (filled ? 1u : 0u);
}
__device__ __forceinline__ bool cell_filled(uint32_t w) { return w & 1u; }
__device__ __forceinline__ int cell_nseg(uint32_t w) { return (int)((w >> 1) & 127u); }
__device__ __forceinline__ int cell_seg_off(uint32_t w) { return (int)(w >> 8); }
// A FILLED cell without occluder pieces ("clean") has no segment offset; its bits 8..31 hold instead its clean
// distance: the Chebyshev distance to the nearest cell that is not clean or lies outside the grid (capped at
// 2^24 - 1; upload_pointmap).  0 for every other cell.  makeGraph's span certificate (makegraph.hip).
constexpr uint32_t CELL_DIST_MAX = (1u << 24) - 1u;
__device__ __forceinline__ int cell_span_dist(uint32_t w) { return ((w & 0xFFu) == 1u) ? (int)(w >> 8) : 0; }

// Run record in HBM: cells from (x0,y0) to (x1,y1) along H, V or a diagonal (PixelVec,
// ngraph.h:31-46).  The direction is implied: y0==y1 -> H, x0==x1 -> V, otherwise diagonal.
struct alignas(8) Run {
    int16_t x0, y0, x1, y1;
};

// Host-mapped control block shared by the host and a running kernel (dmx_ctx_set_progress /
// dmx_ctx_cancel): the host raises `cancel`, workers stop taking work items; workers publish the index
// of the item they took in `progress`.  The reference's Communicator polls IsCancelled and posts the
// record count every 500 ms (genlib/comm.h:59-142, salalib/pointdata.cpp:1301-1316).
struct DmxCtl {
    int cancel;
    int progress;
};
constexpr int CTL_STOP = 1 << 29;   // work index handed out after a cancel: past every range

// Poll at a work grab (one lane): publish the grabbed index every 8th grab, read the cancel word.
// Both are vector memory operations at system scope on host-mapped memory.
__device__ __forceinline__ int ctl_poll(DmxCtl* c, int w) {
    if (!c) return w;
    if ((w & 7) == 0) __hip_atomic_store(&c->progress, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (__hip_atomic_load(&c->cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) return CTL_STOP;
    return w;
}

// Merge links (getMergePixel, vgavisualglobal.cpp:113-122, vgavisualglobaldepth.cpp:55-63): when a cell
// is expanded at level L, its merge partner -- unless already visited -- is extracted at level L as well
// and marked done without being counted.  With every cell of a level expanded (radius n, or a level
// below the radius; context-filled merge cells are refused by the host where they would not expand),
// the outcome does not depend on the pop order inside the level: per link, exactly one end is counted,
// at the level the first end is discovered, and both ends' runs feed the next level.  So after level L
// is published in the frontier F (its cells are new and expandable), for each link (a, b):
//   a and b both in F: both were discovered at L, one of them is not counted (mcorr);
//   one end in F, the other not yet visited: the other joins F and V at L, uncounted (cell_level = L
//   in seed mode); a partner that is discoverable at all counts towards the early-exit total (mdisc).
// The BFS kernels pre-set V with the never-discoverable seed cells, so "visited" is V without them.
// Tiled bitmaps: word (y >> 3) * tw + (x >> 3), bit (y & 7) * 8 + (x & 7); V in LDS (v_lds) or in
// per-workgroup HBM; Fsr / Fsc: optional per-tile frontier summaries of vga_tile.hip.
__device__ __forceinline__ void merge_level_pass(const int2* mpairs, int nmp, int rows, int tw, int ntpb,
                                                 unsigned long long* F, unsigned long long* V, bool v_lds,
                                                 const unsigned long long* seed_tiles, unsigned long long* Fsr,
                                                 unsigned long long* Fsc, int wr, int wc, int32_t* cell_level,
                                                 int lev, unsigned long long* mcorr, unsigned long long* mdisc,
                                                 unsigned long long* mass) {
    for (int i = threadIdx.x; i < nmp; i += ntpb) {
        const int2 pr = mpairs[i];
        const int ax = pr.x / rows, ay = pr.x % rows, bx = pr.y / rows, by = pr.y % rows;
        const int at = (ay >> 3) * tw + (ax >> 3), bt = (by >> 3) * tw + (bx >> 3);
        const unsigned long long ab = 1ull << ((ay & 7) * 8 + (ax & 7)), bb = 1ull << ((by & 7) * 8 + (bx & 7));
        const bool fa = (F[at] & ab) != 0ull, fb = (F[bt] & bb) != 0ull;
        if (fa && fb) {
            atomicAdd(mcorr, 1ull);
        } else if (fa || fb) {
            const int ot = fa ? bt : at;
            const unsigned long long ob = fa ? bb : ab;
            const bool seed = (seed_tiles[ot] & ob) != 0ull;
            const unsigned long long vw =
                v_lds ? V[ot] : __hip_atomic_load(&V[ot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (seed || !(vw & ob)) {
                atomicOr(&F[ot], ob);
                if (v_lds) atomicOr(&V[ot], ob);
                else __hip_atomic_fetch_or(&V[ot], ob, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (Fsr) {
                    const int tx = ot % tw, ty = ot / tw;
                    atomicOr(&Fsr[ty * wr + (tx >> 6)], 1ull << (tx & 63));
                    if (Fsc) atomicOr(&Fsc[tx * wc + (ty >> 6)], 1ull << (ty & 63));
                }
                if (cell_level) cell_level[(size_t)ot * 64 + __ffsll((long long)ob) - 1] = lev;
                if (!seed) atomicAdd(mdisc, 1ull);
                atomicAdd(mass, 1ull);
            }
        }
    }
}

// Merge links with one end context-filled at an odd PixelRef (a, not expanded under a radius) and the
// other end b expandable.  When a source discovers both at the same level L (< radius), the reference's
// outcome depends on which it pops first (vgavisualglobal.cpp:99-122): b first extracts a (a is not
// counted, its runs feed L + 1); a first counts a and leaves it unexpanded.  The level-synchronous BFS
// cannot tell, so such a source raises KERR_ORDER and is marked in oflag[src]: the host re-runs it in the
// reference's own order (vga_ordered.hip).  In every other case the merge pass above is exact: a
// new at L is not in F (not expanded) and so extracts nothing, and b extracts an unvisited a into F.
// Called after the merge pass of level L (F: the expandable cells new at L; V includes every cell new at
// L).  mamb[k] = (a, b); mseen[k] (per workgroup, thread k's own slot across levels) holds the stamp of the
// source for which a was found, so "a in V and not yet seen" means a is new at this level (the check runs
// at every level from 1; a cell in V at level 0 -- a merge partner of the source -- has its partner at
// level 0, not in F).  A cell never discoverable by runs (seed) is only ever reached through its link.
__device__ __forceinline__ void merge_order_check(const int2* mamb, int nmamb, int rows, int tw, int ntpb,
                                                  const unsigned long long* F, const unsigned long long* V,
                                                  bool v_lds, const unsigned long long* seed_tiles, int32_t* mseen,
                                                  int32_t stamp, int* error, uint8_t* oflag, int64_t src) {
    for (int k = threadIdx.x; k < nmamb; k += ntpb) {
        if (mseen[k] == stamp) continue;
        const int2 pr = mamb[k];
        const int ax = pr.x / rows, ay = pr.x % rows, bx = pr.y / rows, by = pr.y % rows;
        const int at = (ay >> 3) * tw + (ax >> 3), bt = (by >> 3) * tw + (bx >> 3);
        const unsigned long long ab = 1ull << ((ay & 7) * 8 + (ax & 7)), bb = 1ull << ((by & 7) * 8 + (bx & 7));
        if (seed_tiles[at] & ab) continue;
        const unsigned long long vw =
            v_lds ? V[at] : __hip_atomic_load(&V[at], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (!(vw & ab)) continue;
        mseen[k] = stamp;
        if ((F[bt] & bb) && !(F[at] & ab)) {
            atomicOr(error, (int)KERR_ORDER);
            oflag[src] = 1;
        }
    }
}

__device__ __host__ __forceinline__ unsigned long long cell_weight(unsigned long long c) {
    unsigned long long z = c * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// direction of a run: 0 along x, 1 along y, 2 along (+1,+1), 3 along (+1,-1); single cells use 0
__device__ __forceinline__ int run_dir(Run ru) {
    if (ru.y0 == ru.y1) return 0;
    if (ru.x0 == ru.x1) return 1;
    return (ru.y1 > ru.y0) ? 2 : 3;
}
__device__ __forceinline__ void dir_step(int dir, int& dx, int& dy) {
    dx = (dir == 1) ? 0 : 1;
    dy = (dir == 0) ? 0 : ((dir == 3) ? -1 : 1);
}

// One run of node u: its share of HO(u) (the prefix-sum difference of the weights along the run's line) and
// the range add of s(u) over the run's cells into the difference arrays D (memory-side atomics).
__device__ __forceinline__ unsigned long long sym_run_scatter(Run ru, unsigned long long su, int cols, int rows,
                                                              const unsigned long long* prefix, unsigned long long* diff) {
    const int64_t C = (int64_t)cols * rows;
    const int dir = run_dir(ru);
    int dx, dy;
    dir_step(dir, dx, dy);
    const int px = ru.x0 - dx, py = ru.y0 - dy, ex = ru.x1 + dx, ey = ru.y1 + dy;
    const unsigned long long* P = prefix + (int64_t)dir * C;
    unsigned long long acc = P[(int64_t)ru.x1 * rows + ru.y1];
    if (px >= 0 && px < cols && py >= 0 && py < rows) acc -= P[(int64_t)px * rows + py];
    unsigned long long* D = diff + (int64_t)dir * C;
    atomicAdd(&D[(int64_t)ru.x0 * rows + ru.y0], su);
    if (ex >= 0 && ex < cols && ey >= 0 && ey < rows) atomicAdd(&D[(int64_t)ex * rows + ey], (unsigned long long)(0ull - su));
    return acc;
}

} // namespace dmx
