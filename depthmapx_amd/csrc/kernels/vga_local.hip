// vga_local.hip -- VGA visual local (-vl): VGAVisualLocal::run (salalib/vgamodules/vgavisuallocal.cpp:23-117).
//
// Per source s with neighbourhood V(s) = the cells of its runs (Node::contents, ngraph.cpp:184-191):
//   cluster  = sum over filled neighbours n of |cells(n) ∩ V(s)|        (int, wraps like the reference)
//   control  = sum over filled neighbours n, in PixelRef order, of 1.0f/float(|cells(n)|)   (float chain)
//   total    = |union of cells(n)|
// and the three columns cluster/(k(k-1)), control, k/total with k = |V(s)| (-1 for k <= 1).
//
// One workgroup per source.  V(s) and the union live in LDS (above ~780^2 cells: in a per-workgroup
// slice of HBM) as 8x8-cell tile bitmaps (the layout of
// vga_tile.hip), so a neighbour's run costs one LDS word per tile it crosses: AND + popcount for the
// intersection, a test-then-OR for the union.  The control sum is a sequential float chain in x-major
// cell order (the reference sorts the neighbourhood): wave 0 walks the columns 64 cells at a time and
// adds the members' terms lane by lane, so the result is the reference's bits.
#include "common.hpp"

namespace dmx {

constexpr int VL_THREADS = 256;

// Visit the tile words a run covers: f(word index, mask of the run's cells in that tile).
template <class F>
__device__ __forceinline__ void run_tile_words(int tw, Run ru, F&& f) {
    if (ru.y0 == ru.y1 && ru.x0 != ru.x1) {
        const int y = ru.y0, rowoff = (y >> 3) * tw, sh = (y & 7) * 8;
        for (int tx = ru.x0 >> 3; tx <= (ru.x1 >> 3); tx++) {
            const int lo = max((int)ru.x0, tx * 8) & 7, hi = min((int)ru.x1, tx * 8 + 7) & 7;
            f(rowoff + tx, (unsigned long long)((0xFFu >> (7 - hi)) & (0xFFu << lo) & 0xFFu) << sh);
        }
    } else if (ru.x0 == ru.x1 && ru.y0 != ru.y1) {
        const int x = ru.x0, tx = x >> 3;
        const unsigned long long col = 0x0101010101010101ull << (x & 7);
        for (int ty = ru.y0 >> 3; ty <= (ru.y1 >> 3); ty++) {
            const int lo = max((int)ru.y0, ty * 8) & 7, hi = min((int)ru.y1, ty * 8 + 7) & 7;
            f(ty * tw + tx, col & (~0ull >> (8 * (7 - hi))) & (~0ull << (8 * lo)));
        }
    } else {
        const int dy = (ru.y1 > ru.y0) ? 1 : -1;
        int x = ru.x0, y = ru.y0;
        while (x <= ru.x1) {
            int n;
            const unsigned long long m = diag_tile_mask(x, y, dy, ru.x1, n);
            f((y >> 3) * tw + (x >> 3), m);
            x += n;
            y += dy * n;
        }
    }
}

// Cells iterated by Node::first/next over a node's runs (Bin::next, ngraph.cpp:399-406).
__global__ void node_size_kernel(int64_t n, const int64_t* node_run_start, const int32_t* node_nruns, const Run* pool,
                                 int32_t* node_size) {
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (k >= n) return;
    const int64_t rs = node_run_start[k];
    const int nr = node_nruns[k];
    int acc = 0;
    for (int r = lane; r < nr; r += 64) {
        const Run ru = pool[rs + r];
        acc += (ru.x0 == ru.x1 && ru.y0 != ru.y1) ? (ru.y1 - ru.y0 + 1) : (ru.x1 - ru.x0 + 1);
    }
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) node_size[k] = acc;
}

// GBM = false: both bitmaps in LDS (grids up to ~780^2 cells); true: a per-workgroup slice of HBM
// scratch (2*tw*th words at gbm + blockIdx.x * 2*nt), L2-resident, for larger grids.
template <bool GBM>
__global__ void __launch_bounds__(VL_THREADS) vga_local_kernel(int cols, int rows, int tw, int th,
                                                               const int32_t* node_cell, const int32_t* cell_node,
                                                               const uint8_t* node_flags, const int64_t* node_run_start,
                                                               const int32_t* node_nruns, const Run* pool,
                                                               const int32_t* node_size, int64_t sb, int64_t se,
                                                               int gates_only, float* out,
                                                               unsigned long long* stats, unsigned long long* gbm) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long vl_lds[];
    const int nt = tw * th;
    unsigned long long* const bm = GBM ? gbm + (size_t)blockIdx.x * 2 * nt : vl_lds;
    unsigned long long* S = bm;        // V(s)
    unsigned long long* U = bm + nt;   // union of the neighbours' cells
    __shared__ long long red_cl[VL_THREADS / 64];
    __shared__ int red_k[VL_THREADS / 64], red_t[VL_THREADS / 64];
    __shared__ float s_control;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int NW = VL_THREADS / 64;
    unsigned long long runs_seen = 0;
    for (int64_t src = sb + blockIdx.x; src < se; src += gridDim.x) {
        float* o = out + src * 3;
        const int c = node_cell[src];
        const int sx = c / rows, sy = c % rows;
        if (((node_flags[src] & 1) && !((sx % 2) == 0 && (sy % 2) == 0)) || gates_only) {
            if (threadIdx.x < 3) o[threadIdx.x] = -1.0f;   // skipped (count only)
            continue;
        }
        for (int t = threadIdx.x; t < 2 * nt; t += VL_THREADS) bm[t] = 0ull;
        __syncthreads();
        {
            const int64_t rs = node_run_start[src];
            const int nr = node_nruns[src];
            for (int r = threadIdx.x; r < nr; r += VL_THREADS)
                run_tile_words(tw, pool[rs + r], [&](int w, unsigned long long m) { atomicOr(&S[w], m); });
        }
        __syncthreads();
        // neighbours: tiles dealt to waves, the cells of a tile in bit order, lanes over each one's runs
        long long cl = 0;
        for (int t = wave; t < nt; t += NW) {
            unsigned long long m = S[t];
            while (m) {
                const int b = __builtin_ctzll(m);
                m &= m - 1;
                const int x = (t % tw) * 8 + (b & 7), y = (t / tw) * 8 + (b >> 3);
                const int nn = cell_node[(int64_t)x * rows + y];
                if (nn < 0) continue;   // not FILLED (a gap cell of a diagonal run)
                const int64_t rs = node_run_start[nn];
                const int nr = node_nruns[nn];
                runs_seen += nr;
                for (int r = lane; r < nr; r += 64)
                    run_tile_words(tw, pool[rs + r], [&](int w, unsigned long long mk) {
                        cl += __popcll(S[w] & mk);
                        if ((U[w] & mk) != mk) atomicOr(&U[w], mk);
                    });
            }
        }
        __syncthreads();
        int k = 0, tot = 0;
        for (int t = threadIdx.x; t < nt; t += VL_THREADS) {
            k += __popcll(S[t]);
            tot += __popcll(U[t]);
        }
        for (int off = 32; off >= 1; off >>= 1) {
            cl += __shfl_xor(cl, off);
            k += __shfl_xor(k, off);
            tot += __shfl_xor(tot, off);
        }
        if (lane == 0) { red_cl[wave] = cl; red_k[wave] = k; red_t[wave] = tot; }
        if (wave == 0) {
            // the reference's float chain over the sorted neighbourhood (x-major cell order)
            float control = 0.0f;
            for (int x = 0; x < cols; x++) {
                const int tcol = x >> 3;
                const unsigned long long xb = 1ull << (x & 7);
                for (int y0 = 0; y0 < rows; y0 += 64) {
                    const int y = y0 + lane;
                    bool mem = false;
                    float term = 0.0f;
                    if (y < rows && (S[(y >> 3) * tw + tcol] & (xb << ((y & 7) * 8)))) {
                        const int nn = cell_node[(int64_t)x * rows + y];
                        if (nn >= 0) {
                            mem = true;
                            term = __fdiv_rn(1.0f, (float)node_size[nn]);
                        }
                    }
                    unsigned long long bal = __ballot(mem);
                    while (bal) {
                        const int l = __builtin_ctzll(bal);
                        bal &= bal - 1;
                        control += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(term), l));
                    }
                }
            }
            if (lane == 0) s_control = control;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            long long clt = 0;
            int kt = 0, tt = 0;
            for (int w = 0; w < NW; w++) { clt += red_cl[w]; kt += red_k[w]; tt += red_t[w]; }
            if (kt > 1) {
                const int32_t cluster = (int32_t)(uint32_t)(unsigned long long)clt;   // int in the reference
                o[0] = (float)((double)cluster / ((double)kt * ((double)kt - 1.0)));
                o[1] = s_control;
                o[2] = (float)((double)kt / (double)tt);
            } else {
                o[0] = o[1] = o[2] = -1.0f;
            }
        }
        __syncthreads();
    }
    if (stats) {
        for (int off = 32; off >= 1; off >>= 1) runs_seen += __shfl_xor(runs_seen, off);
        if (lane == 0) atomicAdd(&stats[0], runs_seen / 64);   // every lane counted each neighbour's runs
    }
}

} // namespace dmx
