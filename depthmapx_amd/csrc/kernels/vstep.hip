// vstep.hip -- visual step depth over the whole GPU, for the maps the tile-resolved BFS does not take
// (grids above 1024^2 cells, or graphs too asymmetric for its bottom-up levels).
//
// VGAVisualGlobalDepth::run (salalib/vgamodules/vgavisualglobaldepth.cpp:23-77) is a multi-source
// BFS: the selected cells are level 0 and always expand; a cell popped at level L > 0 takes the
// value L and expands unless it is context-filled at an odd PixelRef (:53); expanding walks the
// node's runs (Node::extractUnseen) and queues every cell not yet seen.  The value of a filled cell is
// its BFS level, whatever the order inside a level (merge links: vsd_merge_kernel), so the search is
// level-synchronous and top-down:
//   - one wave per frontier node, lanes over its runs;
//   - a run is walked tile word by tile word (8x8-cell words, the layout of vga_tile.hip) against
//     the visited bitmap: atomicOr claims the unseen cells of the word, each newly seen cell takes
//     level L+1, and the expandable filled ones join the next frontier.
// Cost: 8 B per run plus one bitmap word per 8 cells of run length, per expanded node.
#pragma once

namespace dmx {

constexpr int VSD_THREADS = 256;

__global__ void __launch_bounds__(VSD_THREADS) vsd_level_kernel(int rows, int tw, const int32_t* frontier, int64_t nf,
                                                                const int64_t* node_run_start, const int32_t* node_nruns,
                                                                const Run* pool, const int32_t* cell_node,
                                                                const uint8_t* node_flags, int next_level,
                                                                unsigned long long* vis, int32_t* level, int32_t* next,
                                                                unsigned long long* next_n) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * (VSD_THREADS / 64);
    for (int64_t f = (int64_t)blockIdx.x * (VSD_THREADS / 64) + (threadIdx.x >> 6); f < nf; f += waves) {
        const int32_t node = frontier[f];
        const int64_t rs = node_run_start[node];
        const int nr = node_nruns[node];
        for (int r = lane; r < nr; r += 64)
            run_tile_words(tw, pool[rs + r], [&](int w, unsigned long long m) {
                if ((vis[w] & m) == m) return;   // all seen (a stale read only costs the atomic below)
                unsigned long long fresh = m & ~atomicOr(&vis[w], m);
                while (fresh) {
                    const int b = __builtin_ctzll(fresh);
                    fresh &= fresh - 1;
                    const int x = (w % tw) * 8 + (b & 7), y = (w / tw) * 8 + (b >> 3);
                    const int64_t c = (int64_t)x * rows + y;
                    level[c] = next_level;
                    const int32_t nn = cell_node[c];
                    // PixelRef::iseven: both coordinates even
                    if (nn >= 0 && (!(node_flags[nn] & 1) || ((x % 2) == 0 && (y % 2) == 0)))
                        next[atomicAdd(next_n, 1ull)] = nn;
                }
            });
    }
}

// PixelRef::iseven: both coordinates even.  A cell popped at a level > 0 expands unless it is
// context-filled at an odd PixelRef (vgavisualglobaldepth.cpp:52).
__device__ __forceinline__ bool vsd_expands(int rows, int c, const int32_t* cell_node, const uint8_t* node_flags) {
    const int x = c / rows, y = c % rows;
    return !(node_flags[cell_node[c]] & 1) || ((x % 2) == 0 && (y % 2) == 0);
}

// Merge links after level L of the search (vgavisualglobaldepth.cpp:55-63), L >= 1:
//  - one end new at L and expanded, the other not yet seen: the other is extracted now -- it takes level L
//    and its node joins the next frontier (whatever its own fill: the partner's node is extracted as is);
//  - one end new at L but not expanded (context-filled, odd): nothing (the reference only looks at the
//    merge pixel of a cell it expands);
//  - both ends new at L: both hold L.  If both or neither expand, nothing else happens.  If exactly one
//    does, the reference extracts the other one's node only when it pops the expanding end first; that
//    node goes on `pend`, and vsd_pending_kernel checks after level L + 1 that extracting it would have
//    found nothing new (then the result is the same in either order).
__global__ void vsd_merge_kernel(int rows, int tw, const int2* mpairs, int nmp, const int32_t* cell_node,
                                 const uint8_t* node_flags, int lev, unsigned long long* vis, int32_t* level,
                                 int32_t* next, unsigned long long* next_n, int32_t* pend, unsigned long long* pend_n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nmp) return;
    const int2 pr = mpairs[i];
    const int la = level[pr.x], lb = level[pr.y];
    if (la != lev && lb != lev) return;
    const bool ea = la == lev && vsd_expands(rows, pr.x, cell_node, node_flags);
    const bool eb = lb == lev && vsd_expands(rows, pr.y, cell_node, node_flags);
    if (la == lev && lb == lev) {
        if (ea != eb) pend[atomicAdd(pend_n, 1ull)] = cell_node[ea ? pr.y : pr.x];
        return;
    }
    const int o = (ea && lb < 0) ? pr.y : ((eb && la < 0) ? pr.x : -1);
    if (o < 0) return;
    const int x = o / rows, y = o % rows;
    atomicOr(&vis[(y >> 3) * tw + (x >> 3)], 1ull << ((y & 7) * 8 + (x & 7)));
    level[o] = lev;
    next[atomicAdd(next_n, 1ull)] = cell_node[o];
}

// The pending extractions of vsd_merge_kernel, once level L + 1 is complete (with its merge links): a
// filled cell on the node's runs that is still unseen would take level L + 1 in one pop order and a later
// level (or none) in the other.  Flags error[0] then.  One wave per node, lanes over its runs.
__global__ void __launch_bounds__(VSD_THREADS) vsd_pending_kernel(int rows, int tw, const int32_t* pend, int64_t np,
                                                                  const int64_t* node_run_start, const int32_t* node_nruns,
                                                                  const Run* pool, const int32_t* cell_node,
                                                                  const unsigned long long* vis, int* error) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * (VSD_THREADS / 64);
    for (int64_t f = (int64_t)blockIdx.x * (VSD_THREADS / 64) + (threadIdx.x >> 6); f < np; f += waves) {
        const int32_t node = pend[f];
        const int64_t rs = node_run_start[node];
        const int nr = node_nruns[node];
        for (int r = lane; r < nr; r += 64)
            run_tile_words(tw, pool[rs + r], [&](int w, unsigned long long m) {
                for (unsigned long long u = m & ~vis[w]; u; u &= u - 1) {
                    const int b = __builtin_ctzll(u);
                    const int x = (w % tw) * 8 + (b & 7), y = (w / tw) * 8 + (b >> 3);
                    if (cell_node[(int64_t)x * rows + y] >= 0) atomicOr(error, (int)KERR_ORDER);
                }
            });
    }
}

} // namespace dmx
