// makegraph.hip -- K1/K2: the spark-sieve inter-visibility sweep + run-length binning on gfx950.
//
// Replaces PointMap::sparkGraph2 / sparkPixel2 / sieve2 (salalib/pointdata.cpp:1246-1341,
// :1380-1565), sparkSieve2 (salalib/sparksieve2.cpp:33-173), whichbin (pointdata.h:432-520),
// Node::make / Bin::make (ngraph.cpp:27-58, :234-304) and addGridConnections (pointdata.cpp:1735).
//
// Decomposition (MI355X-first, not the reference's per-pixel std::set loop):
//   * one wavefront owns one source cell at a time (persistent grid, dynamic source counter);
//     the 8 octants run in reference order q = 0..7 so the FP64 moment sums keep their order;
//   * inside an octant the depth loop is sequential (each depth's gaps depend on the previous),
//     but the candidate cells of one depth are spread over the 64 lanes: per-gap index ranges and
//     the reference's monotone `firstind` rule become a prefix-max + prefix-sum over the gap list;
//   * the gap list, the per-depth block list and per-row run state live in LDS;
//   * visible cells never go through a sort: each octant row (fixed `ind`) is walked in depth
//     order, so runs are closed incrementally per row; a per-(bin,row) count array gives every run
//     its final slot in reference (PixelRefH/V) order without sorting (counting placement);
//   * runs are staged per wave in scratch, then copied once into a global pool reserved with one
//     atomic per source, bins in reference order 0..31; a whole-graph build also does the VGA
//     symmetry certificate's scatter there (sym_run_scatter, common.hpp), run by run.
//   All geometry is IEEE double in the reference's operation order (-ffp-contract=off).
#include "common.hpp"
#include "span.hpp"


namespace dmx {

#ifndef MK_PFIND
#define MK_PFIND 1   // the prefetch also keeps the first chunk's candidate index and gap bounds in registers (A/B hook)
#endif
// span A/B hooks, configs[2] / configs[4] makeGraph seconds on one box (profiles/r6_span_ab2.jsonl; off: 3.118 / 8.692):
#ifndef MK_SPAN_CB
#define MK_SPAN_CB 0      // the classes some lane has from 5 ballots instead of two wave max scans: 3.245 / 8.880
#endif
#ifndef MK_SPAN_GSKIP
#define MK_SPAN_GSKIP 1   // skip a gap no row of the chunk can see over the span: 2.948 / 8.458
#endif
#ifndef MK_WFRED
#define MK_WFRED 0        // span integer wave max / min through the DPP whole-wave reductions: 3.020 / 8.365 (gl 2.877 / 8.251)
#endif
#ifndef MK_SPAN_RCP
#define MK_SPAN_RCP 0     // span row estimates from v_rcp_f64 instead of divisions (settled exactly either way): 2.886 / 8.237
#endif
#ifndef MK_SPAN_LSUM
#define MK_SPAN_LSUM 1    // span counts (visible, examined) kept per lane, reduced once per source: 3.060 / 8.423
#endif
constexpr int MK_GCAP0 = 16, MK_BCAP0 = 32;   // first-pass LDS gap / block capacities (FIXED kernels)
// shortest occluder-free span taken, in depths (DMX_MK_SPAN overrides): configs[2] / configs[4] makeGraph with
// 1: 3.23 / 9.61 s, 2: 3.17 / 9.02, 4: 3.11 / 8.61, 8: 3.11 / 8.75 (profiles/r6_span_ab.jsonl); with the gap skip
// 3: 2.884 / 8.261, 4: 2.886 / 8.244, 5: 2.881 / 8.255, 6: 2.889 / 8.306 (r6_span_ab2.jsonl, tags s3..s6)
constexpr int MK_SPAN_MIN = 4;
// open-run state of rows 0 .. MK_OPEN_LDS-1 lives in LDS, of farther rows (grids above ~1020 cells a
// side) in per-wave scratch memory: rows past 1024 are reached only by sight lines longer than 1024
// cells, and a full-length LDS array would cost a 2000^2 grid a quarter of its waves
constexpr int MK_OPEN_LDS = 1024;
constexpr int64_t MK_CAPACITY_TAG = 1ll << 62, MK_NODE_MASK = MK_CAPACITY_TAG - 1;
// symmetry adjacency bits: open-run state, emission record (shallow / deep end adjacent), staged run (bit 14
// of x0 / x1: the start / end range add cancels; grids below 16384 cells a side)
constexpr uint32_t MK_OPEN_ADJ = 0x80000000u;
constexpr int MK_REC_SHALLOW = 58, MK_REC_DEEP = 59;
constexpr int16_t MK_RUN_FLAG = 0x4000;

struct MakeGraphParams {
    int cols, rows;
    double spacing, blx, bly;
    double maxdist;
    const uint32_t* cellw;     // [C] packed cell word (common.hpp)
    double sqrt_err;
    const double* segs;        // [S][4] cropped segment start/end
    const int32_t* node_cell;  // [N] node -> x-major cell index
    int64_t node_begin, node_end;
    int* work_counter;         // dynamic source counter (zeroed by the host each launch)
    DmxCtl* ctl;               // host-mapped progress / cancel block (nullptr: none)
    unsigned long long* pool_cursor;
    int64_t pool_capacity;     // in runs
    Run* pool;
    int64_t* node_run_start;   // [N] (indexed by node - node_begin)
    int32_t* bin_nruns;        // [N][32]
    uint16_t* bin_count;       // [N][32]
    float* bin_dist;           // [N][32]
    float* attrs;              // [N][3]
    unsigned long long* stageA;  // per wave: capA packed emission records
    Run* stageB;               // per wave: capB runs (canonical octant segments)
    uint32_t* prefix;          // per wave: 3*(D+1)+2 counts/prefix
    uint32_t* runcnt;          // per wave: 3*(D+1)+1 runs per (slot, row) of the octant (zero between octants)
    int capA, capB;
    int gcap, bcap;            // LDS gap / block capacities
    double2* bspill;           // per wave: [2][spill_cap] blocks past bcap (raw, sorted)
    int* bspill_flag;          // per wave: [spill_cap]
    int spill_cap;
    int dmax;                  // max(cols, rows)
    int* error;
    unsigned long long* stats; // [0] sieve cells examined, [1] visible (source, target) pairs
    // retry mode: process node_list[0, list_n) instead of [node_begin, node_end); sources that
    // exceed a capacity are appended to fail_list and re-run by the host with larger capacities
    const int64_t* node_list;
    int64_t list_n;
    int64_t* fail_list;
    int* fail_count;
    int profile;               // 1: accumulate per-phase clocks into stats[8..13]
    int exact_moments;         // 1: the reference's serial FP64 moment chains; 0: certified parallel sums
    uint32_t* src_work;        // optional [n][2]: depth steps and candidate chunks of each published source
    uint32_t* openh;           // per wave: open-run state of rows >= MK_OPEN_LDS (zeroed by the host, kept zero)
    int openh_n;               // its length per wave: max(0, dmax + 4 - MK_OPEN_LDS)
    // the VGA symmetry certificate's scatter, done as each source publishes its runs (null: off; vga_do.hip
    // prepare_symmetry then scans the pool): HO per node and the range adds of s(u) along each run's line
    const unsigned long long* sym_prefix;   // [4][C] line prefix sums of the cell weights
    unsigned long long* sym_diff;           // [4][C] difference arrays (zeroed by the host per pass)
    unsigned long long* sym_ho;             // [N] (indexed by node - node_begin)
    // occluder-free depth spans (span.hpp): the shortest span taken, in depths (0: off); the cell words of FILLED
    // cells without an occluder piece carry their clean distance (common.hpp cell_span_dist)
    int spans;
};

// phase clocks (profile builds of a run only; wave-uniform scalar reads)
#define MK_T(i)                                                           \
    if (PROF) {                                                           \
        const unsigned long long n_ = __builtin_amdgcn_s_memtime();       \
        cyc[i] += n_ - tmark;                                             \
        tmark = n_;                                                       \
    }

// ------------------------------------------------------------------ octant tables
// q octants (sparksieve2.cpp:134-141):   \ 6 | 7 /   0 \ | / 1   2 / | \ 3   / 4 | 5 \ .
__constant__ int c_sector_base[8] = {13, 1, 17, 29, 21, 25, 9, 5};
__constant__ int c_axis_bin[8] = {16, 0, -1, -1, -1, 24, 8, -1};
__constant__ int c_diag_bin[8] = {12, 4, 20, 28, -1, -1, -1, -1};
// canonical (PixelRefH: y then x / PixelRefV: x then y) order expressed in (ind, depth)
__constant__ int c_row_asc[8] = {1, 1, 0, 0, 0, 1, 0, 1};
__constant__ int c_d_asc[8] = {0, 1, 0, 1, 0, 0, 1, 1};
// 1 if the octant's axis / diagonal bin sorts before its sectors (lower bin number)
__constant__ int c_axis_low[8] = {0, 1, 0, 0, 0, 1, 1, 0};
__constant__ int c_diag_low[8] = {1, 0, 0, 1, 0, 0, 0, 0};
// the order in which octant segments are laid out so bins come out 0..31 (Node::make order)
__constant__ int c_seg_order[8] = {1, 7, 6, 0, 2, 4, 5, 3};

__device__ __forceinline__ void octant_cell(int q, int cx, int cy, int depth, int ind, int& hx, int& hy) {
    int x = (q >= 4 ? ind : depth);
    int y = (q >= 4 ? depth : ind);
    hx = (short)(cx + ((q & 1) ? x : -x));                // pointdata.cpp:1536-1540
    hy = (short)(cy + ((q <= 1 || q >= 6) ? y : -y));
}

// sparkSieve2::tanify (sparksieve2.cpp:143-173)
__device__ __forceinline__ double tanify(double cxp, double cyp, double px, double py, int q) {
    switch (q) {
    case 0: return (py - cyp) / (cxp - px);
    case 1: return (py - cyp) / (px - cxp);
    case 2: return (cyp - py) / (cxp - px);
    case 3: return (cyp - py) / (px - cxp);
    case 4: return (cxp - px) / (cyp - py);
    case 5: return (px - cxp) / (cyp - py);
    case 6: return (cxp - px) / (py - cyp);
    default: return (px - cxp) / (py - cyp);
    }
}

// whichbin (pointdata.h:432-520): span.hpp (shared with the span arithmetic and its host test)

// block zone ordering (sparksieve2.h:72-75)
__device__ __forceinline__ bool zone_less(double as, double ae, double bs, double be) {
    return (as == bs) ? (ae > be) : (as < bs);
}

__device__ __forceinline__ unsigned long long ballot(bool p) { return __ballot(p); }
// lane j's double (j wave-uniform)
__device__ __forceinline__ double readlane_d(double v, int j) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), j), __builtin_amdgcn_readlane(__double2loint(v), j));
}
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int prefix_popc(unsigned long long m) {
    return __popcll(m & ((1ull << lane_id()) - 1ull));
}

// wave-wide inclusive scans over 64 lanes (int)
__device__ __forceinline__ int wave_incl_sum(int v) {
    for (int o = 1; o < 64; o <<= 1) {
        int t = __shfl_up(v, o);
        if (lane_id() >= o) v += t;
    }
    return v;
}
__device__ __forceinline__ int wave_incl_max(int v) {
    for (int o = 1; o < 64; o <<= 1) {
        int t = __shfl_up(v, o);
        if (lane_id() >= o) v = max(v, t);
    }
    return v;
}
// max over all 64 lanes (every lane gets it)
// (all 64 lanes active at every call)
__device__ __forceinline__ int wave_incl_max_all(int v) {
#if MK_WFRED
    return __ockl_wfred_max_i32(v);
#else
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
#endif
}
__device__ __forceinline__ double wave_max_d(double v) {
    for (int o = 32; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}

// emission record: slot(2) | ind(14) | dstart(14) | dend(14) | k(14)
__device__ __forceinline__ unsigned long long pack_emit(int slot, int ind, int ds, int de, int k) {
    return (unsigned long long)slot | ((unsigned long long)ind << 2) | ((unsigned long long)ds << 16) |
           ((unsigned long long)de << 30) | ((unsigned long long)k << 44);
}

// Symmetry range adds of one published run (common.hpp sym_run_scatter) with two changes the in-hash does not
// see: a single cell takes its octant's direction (x for H octants, y for V: its prefix sum is the cell
// whatever the direction), so a run and its neighbour in the row share one difference array; and the ends
// flagged by the sweep (a run ending where the row's next run starts) skip the +s / -s pair that cancels.
__device__ __forceinline__ unsigned long long sym_run_scatter_q(Run ru, int q, bool skip0, bool skip1, unsigned long long su,
                                                                int cols, int rows, const unsigned long long* prefix,
                                                                unsigned long long* diff) {
    const int64_t C = (int64_t)cols * rows;
    const int dir = (ru.x0 == ru.x1 && ru.y0 == ru.y1) ? (q < 4 ? 0 : 1) : run_dir(ru);
    int dx, dy;
    dir_step(dir, dx, dy);
    const int px = ru.x0 - dx, py = ru.y0 - dy, ex = ru.x1 + dx, ey = ru.y1 + dy;
    const unsigned long long* Pf = prefix + (int64_t)dir * C;
    unsigned long long acc = Pf[(int64_t)ru.x1 * rows + ru.y1];
    if (px >= 0 && px < cols && py >= 0 && py < rows) acc -= Pf[(int64_t)px * rows + py];
    unsigned long long* Df = diff + (int64_t)dir * C;
    if (!skip0) atomicAdd(&Df[(int64_t)ru.x0 * rows + ru.y0], su);
    if (!skip1 && ex >= 0 && ex < cols && ey >= 0 && ey < rows) atomicAdd(&Df[(int64_t)ex * rows + ey], (unsigned long long)(0ull - su));
    return acc;
}

// Run for (ind, depth range) in octant q; H octants (q<4) run along x, V octants along y.
__device__ __forceinline__ Run make_run(int q, int cx, int cy, int ind, int ds, int de) {
    int ax, ay, bx, by;
    octant_cell(q, cx, cy, ds, ind, ax, ay);
    octant_cell(q, cx, cy, de, ind, bx, by);
    Run r;
    if (q < 4) { // horizontal: start is the smaller x
        if (ax <= bx) { r.x0 = ax; r.y0 = ay; r.x1 = bx; r.y1 = by; }
        else { r.x0 = bx; r.y0 = by; r.x1 = ax; r.y1 = ay; }
    } else {     // vertical: start is the smaller y
        if (ay <= by) { r.x0 = ax; r.y0 = ay; r.x1 = bx; r.y1 = by; }
        else { r.x0 = bx; r.y0 = by; r.x1 = ax; r.y1 = ay; }
    }
    return r;
}

// One wave per workgroup: lanes exchanging data through LDS need only an ordering point (the wave's LDS
// instructions execute in order); __syncthreads would also drain every outstanding global load and
// store (vmcnt(0)) several times per depth.  Exchanges through global memory keep __syncthreads.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// per-wave counters in HBM scratch (one wave per workgroup reads back its own stores: workgroup scope keeps
// them in L1/L2; agent scope would write every store through to memory and miss L2 on every load)
__device__ __forceinline__ uint32_t ld_l2(const uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void st_l2(uint32_t* p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

// open-run state per row: valid(1) | slot(2) | start(14) | last(14) | adjacent(1): the run started where the
// row's previous run ended (MK_OPEN_ADJ)
__device__ __forceinline__ uint32_t pack_open(int slot, int s, int l) {
    return 1u | ((uint32_t)slot << 1) | ((uint32_t)s << 3) | ((uint32_t)l << 17);
}

// ---- certified moment sums
// The reference accumulates sum(d) and sum(d*d) as two serial FP64 chains in addlist order
// (pointdata.cpp:1490-1495) and stores them as floats.  The fast path sums each lane's share in
// double-double (error-free TwoSum), reduces the wave, and bounds the serial chain's rounding error
// by gamma_(n-1) * sum (non-negative summands): when every double within that bound rounds to the
// same float, that float IS the reference's value.  Otherwise the source is re-run with the serial
// chains (exact_moments), which happens for ~0.2 % of sources at 1000^2.
__device__ __forceinline__ void dd_add(double& h, double& l, double v) {
    const double s = h + v;
    const double bb = s - h;
    l += (h - (s - bb)) + (v - bb);
    h = s;
}
__device__ __forceinline__ void dd_merge(double& h, double& l, double bh, double bl) {
    const double s = h + bh;
    const double bb = s - h;
    const double e = (h - (s - bb)) + (bh - bb);
    const double t = (l + bl) + e;
    h = s + t;
    l = t - (h - s);
}
// Plain per-lane double sums reduced by a 6-level butterfly: |S~ - S| <= gamma_(m+6) S with m the
// largest per-lane count; the reference's serial chain is within gamma_(n-1) S of S.
__device__ __forceinline__ bool certified_float_sum(double S, long long n, long long m, float* out) {
    const double u = 0x1p-53;
    const double g1 = (double)n * u / (1.0 - (double)n * u);
    const double g2 = (double)(m + 7) * u / (1.0 - (double)(m + 7) * u);
    const double E = 2.0 * (g1 + g2) * S + S * 0x1p-50;
    const float a = (float)(S - E), b = (float)(S + E);
    *out = a;
    return a == b;
}
__device__ __forceinline__ bool certified_float(double h, double l, long long n, float* out) {
    const double u = 0x1p-53;
    const double g = (double)n * u / (1.0 - (double)n * u);
    const double E = 2.0 * g * h + 2.0 * fabs(l) + h * 0x1p-50;
    const float a = (float)(h - E), b = (float)(h + E);
    *out = a;
    return a == b;
}

// The float of S when every double within E of S rounds to it (then it is the float of any sum within E).
__device__ __forceinline__ bool certified_float_e(double S, double E, float* out) {
    const float a = (float)(S - E), b = (float)(S + E);
    *out = a;
    return a == b;
}

// Square roots of the moment sums: v_rsq_f64 (~2^-23 relative) and one Newton step (5 FP64
// instructions; the error, ~2^-44, is measured exhaustively over the integers the kernel feeds it by
// sqrt_err_kernel and bounds the certificate) instead of the correctly rounded expansion (~17 instructions).
__device__ __forceinline__ double sqrt_nr(double x) {   // x >= 1
    const double r = __builtin_amdgcn_rsq(x);
    const double g = x * r, h = 0.5 * r;
    return fma(fma(-g, g, x), h, g);
}

// max over n in [1, nmax] of |sqrt_nr(n) - sqrt(n)| / sqrt(n), as the bits of a non-negative double
__global__ void sqrt_err_kernel(long long nmax, unsigned long long* err_bits) {
    double e = 0.0;
    for (long long n = 1 + (long long)blockIdx.x * blockDim.x + threadIdx.x; n <= nmax;
         n += (long long)gridDim.x * blockDim.x) {
        const double x = (double)n, r = sqrt(x), h = sqrt_nr(x);
        e = fmax(e, fabs(h - r) / r);
    }
    for (int off = 32; off >= 1; off >>= 1) e = fmax(e, __shfl_xor(e, off));
    if ((threadIdx.x & 63) == 0) atomicMax(err_bits, (unsigned long long)__double_as_longlong(e));
}

struct Lds {
    double2* gaps;    // [gcap]
    double2* gaps2;   // [gcap] merge output
    double2* blocks;  // [bcap]
    int* ga;          // [gcap] first visited ind per gap
    int2* gc;         // [gcap] centregap ind range per gap: ceil(fl(start*depth)), floor(fl(end*depth))
    int* gpre;        // [gcap+1] exclusive prefix of visited counts
    uint32_t* openr;  // [min(dmax + 4, MK_OPEN_LDS)]
    unsigned* binc;   // [32] node counts per bin
    unsigned* bfar;   // [32] far distance (float bits)
    int* bnr;         // [32] runs per bin
    int* misc;        // [32] scalars: 0 ng, 1 nb, 16..23 segment start, 24..31 segment length
    double2* bsorted; // [bcap] sort output
    int* bflag;       // [bcap] first-occurrence flags
};

// WPE: waves per SIMD the register allocation targets; PROF: per-phase clocks (DMX_VERBOSE builds of
// a run) -- a template flag so that the 8 clock counters cost no registers otherwise
// FIXED: the first pass's LDS capacities (gcap 16, bcap 32) as constants, so the LDS arrays sit at constant
// offsets instead of holding 13 SGPRs (the kernel's time follows its register allocation: spills go to
// scratch memory on the depth loop's critical path); re-runs with larger capacities take FIXED = false.
// COUNT: count each source's depth steps and candidate chunks (the cost sample of dmx_makegraph_balance;
// two more live counters cost the main pass ~10 % through the register allocation, so only the sample
// pass carries them).
// MAXD (FIXED kernels): maxdist != -1 (the maxdist test compiled in).  FAR (FIXED kernels): the grid has
// rows past MK_OPEN_LDS (the scratch-memory branch of the open-run accessors compiled in).
template <int WPE, bool PROF, bool FIXED, bool COUNT, bool MAXD, bool FAR>
// The parameters are read through a pointer to device memory rather than passed by value: the compiler
// then reloads cold fields with scalar loads instead of keeping ~50 pointers live in SGPRs and
// spilling them (VGA tile kernel: 210 -> 105 SGPR spills).
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) makegraph_kernel(const MakeGraphParams* __restrict__ PP) {
    const DMX_CONST_AS MakeGraphParams& P = const_params(PP);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = lane_id();
    const int gcap = FIXED ? MK_GCAP0 : P.gcap, bcap = FIXED ? MK_BCAP0 : P.bcap, D = P.dmax;
    // FIXED kernels run the first pass: certified moment sums, maxdist test only in the MAXD variant
    const bool exact = FIXED ? false : (P.exact_moments != 0);
    const bool hasmax = FIXED ? MAXD : (P.maxdist != -1.0);
    // spans need the certified parallel moment sums (the serial chains sum in the reference's per-depth
    // addlist order) and no maxdist test
    const bool spans = !exact && !hasmax && P.spans > 0;
    const int span_min = P.spans;   // shortest span taken (depths)
    Lds L;
    {
        unsigned char* p = smem;
        L.gaps = (double2*)p; p += sizeof(double2) * gcap;
        L.gaps2 = (double2*)p; p += sizeof(double2) * gcap;
        L.blocks = (double2*)p; p += sizeof(double2) * bcap;
        L.binc = (unsigned*)p; p += 4 * 32;
        L.bfar = (unsigned*)p; p += 4 * 32;
        L.bnr = (int*)p; p += 4 * 32;
        L.misc = (int*)p; p += 4 * 32;
        L.bsorted = (double2*)p; p += sizeof(double2) * bcap;
        L.gc = (int2*)p; p += 8 * gcap;   // (8-aligned: follows the 16-byte arrays)
        L.ga = (int*)p; p += 4 * gcap;
        L.bflag = (int*)p; p += 4 * bcap;
        L.gpre = (int*)p; p += 4 * (gcap + 4);
        L.openr = (uint32_t*)p; p += 4 * min(D + 4, MK_OPEN_LDS);
    }
    const int wave_global = blockIdx.x;
    auto stA = P.stageA + (size_t)wave_global * P.capA;
    auto stB = P.stageB + (size_t)wave_global * P.capB;
    auto spill = P.bspill + (size_t)wave_global * 2 * P.spill_cap;   // [raw | sorted]
    auto spill_flag = P.bspill_flag + (size_t)wave_global * P.spill_cap;
    auto put_block = [&](int i, double2 v) {
        if (i < bcap) L.blocks[i] = v;
        else if (i - bcap < P.spill_cap) spill[i - bcap] = v;
    };
    auto get_block = [&](int i) -> double2 { return i < bcap ? L.blocks[i] : spill[i - bcap]; };
    auto set_flag = [&](int i, int f) {
        if (i < bcap) L.bflag[i] = f;
        else spill_flag[i - bcap] = f;
    };
    auto get_flag = [&](int i) -> int { return i < bcap ? L.bflag[i] : spill_flag[i - bcap]; };
    auto put_sorted = [&](int i, double2 v) {
        if (i < bcap) L.bsorted[i] = v;
        else spill[P.spill_cap + i - bcap] = v;
    };
    auto get_sorted = [&](int i) -> double2 { return i < bcap ? L.bsorted[i] : spill[P.spill_cap + i - bcap]; };
    auto pref = P.prefix + (size_t)wave_global * (3 * (D + 1) + 4);
    auto rcnt = P.runcnt + (size_t)wave_global * (3 * (D + 1) + 4);   // zeroed by the host
    const double sp = P.spacing;
    // the fused symmetry scatter's adjacency flags ride in bit 14 of the staged runs' x coordinates
    const bool symflags = P.sym_diff != nullptr && P.cols < 16384 && P.rows < 16384;

    // LDS state that persists across sources is reset here once
    const int AX = 3 * (D + 1); // rcnt[AX] counts the runs of the axis row (ind 0)
    auto openh = P.openh + (size_t)wave_global * P.openh_n;
    const bool far_rows = FIXED ? FAR : (D + 4 > MK_OPEN_LDS);
    auto ld_open = [&](int i) -> uint32_t {
        return (!far_rows || i < MK_OPEN_LDS) ? L.openr[i] : ld_l2(&openh[i - MK_OPEN_LDS]);
    };
    auto st_open = [&](int i, uint32_t v) {
        if (!far_rows || i < MK_OPEN_LDS) L.openr[i] = v;
        else st_l2(&openh[i - MK_OPEN_LDS], v);
    };
    for (int i = lane; i < min(D + 4, MK_OPEN_LDS); i += 64) L.openr[i] = 0;
    __syncthreads();
    // 0 collectgarbage, 1 visit ranges, 2 candidate tests + blocks, 3 visible: bins, 4 visible: serial
    // moments, 5 visible: run tracking, 6 octant flush + placement, 7 publish, 8 depth tail (next depth's
    // prefetch), 9 octant setup + depth 0
    // (10: spans, outside 11 its rows' class ends and open state, 12 the per-gap depth searches, 13 the per-class pieces)
    unsigned long long cyc[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long mst[4] = {0, 0, 0, 0};   // PROF: merges, one-block merges, blocks, gaps at merges
    unsigned long long spst[6] = {0, 0, 0, 0, 0, 0};   // PROF: spans, span depths, span cells, row chunks, (chunk, gap)
                                                       // pairs, pairs with no visible row
    unsigned long long tmark = PROF ? __builtin_amdgcn_s_memtime() : 0;

    for (;;) {
        int s_idx = 0;
        if (lane == 0) s_idx = ctl_poll(P.ctl, atomicAdd(P.work_counter, 1));
        s_idx = __shfl(s_idx, 0);
        int64_t node;
        if (P.node_list) {
            if (s_idx >= P.list_n) break;
            node = P.node_list[s_idx] & MK_NODE_MASK;
        } else {
            node = P.node_begin + s_idx;
            if (node >= P.node_end) break;
        }
        const int cell = P.node_cell[node];
        // wave-uniform: in scalar registers (held in VGPRs they were spilled around the candidate loop)
        const int cx = __builtin_amdgcn_readfirstlane(cell / P.rows), cy = __builtin_amdgcn_readfirstlane(cell % P.rows);
        const double c0x = P.blx + sp * 1.0 * (double)cx, c0y = P.bly + sp * 1.0 * (double)cy;
        if (lane < 32) { L.binc[lane] = 0; L.bfar[lane] = 0; L.bnr[lane] = 0; }
        __syncthreads();

        double tsum = 0.0, tsum2 = 0.0; // wave-uniform, reference order (exact_moments)
        double s1 = 0.0, s2 = 0.0;   // per-lane sums (fast path, certified at the end)
        unsigned long long s2n = 0;  // per-lane sum of dx^2 + dy^2 (exact)
        int mcnt = 0;                // this lane's summand count
        int nsize = 0;
        unsigned long long examined = 0;
#if MK_SPAN_LSUM
        int nsize_l = 0;                    // this lane's share of the spans' visible cells / cells examined
        unsigned long long examined_l = 0;
#endif
        uint32_t nsteps = 0, nchunks = 0;   // sieve depth steps / 64-candidate chunks (the source's work)
        int bpos = 0;        // next free run slot in stageB
        bool failed = false;
        bool certfail = false;

        const uint32_t own = P.cellw[cell];
        const int own_n = cell_nseg(own), own_off = cell_seg_off(own);

        for (int q = 0; q < 8; q++) {
            // ---- depth 0: own-cell segments cropped to the quarter viewport (pointdata.cpp:1399-1450)
            const double border = sp * 1e-10;
            Rect vp{P.blx + sp * ((double)cx - 0.5 - 1e-10), P.bly + sp * ((double)cy - 0.5 - 1e-10),
                    P.blx + sp * ((double)cx + 0.5 + 1e-10), P.bly + sp * ((double)cy + 0.5 + 1e-10)};
            switch (q) {
            case 0: vp.trx = c0x; vp.bly = c0y - border; break;
            case 6: vp.trx = c0x + border; vp.bly = c0y; break;
            case 1: vp.blx = c0x; vp.bly = c0y - border; break;
            case 7: vp.blx = c0x - border; vp.bly = c0y; break;
            case 2: vp.trx = c0x; vp.tr_y = c0y + border; break;
            case 4: vp.trx = c0x + border; vp.tr_y = c0y; break;
            case 3: vp.blx = c0x; vp.tr_y = c0y + border; break;
            case 5: vp.blx = c0x - border; vp.tr_y = c0y; break;
            }
            if (lane == 0) { L.misc[0] = 1; L.misc[1] = 0; }
            if (lane == 0) L.gaps[0] = make_double2(0.0, 1.0);
            __syncthreads();
            for (int i = lane; i < own_n; i += 64) {
                const double* sg = P.segs + 4 * (size_t)(own_off + i);
                Seg l = make_seg(Vec2{sg[0], sg[1]}, Vec2{sg[2], sg[3]});
                if (clip_seg(l, vp)) {
                    Vec2 a = l.start(), b = l.end();
                    double ta = tanify(c0x, c0y, a.x, a.y, q), tb = tanify(c0x, c0y, b.x, b.y, q);
                    const int slot = atomicAdd(&L.misc[1], 1);
                    put_block(slot, (ta < tb) ? make_double2(ta - 1e-10, tb + 1e-10) : make_double2(tb - 1e-10, ta + 1e-10));
                }
            }
            __syncthreads();

            int ng = 1;
            int dq = 0;                 // deepest depth visited in this octant
            int diag_n = 0, diag_min = 0, diag_max = 0;
            int nA = 0;                 // emissions staged in this octant
            const int q_sector = c_sector_base[q], q_axis = c_axis_bin[q], q_diag = c_diag_bin[q];
            // whichbin of this octant's directions by ratio class: axis, < tan15, < tan30, < 1, diagonal
            unsigned obinp = 0;   // 6 bits a class
            {
                const double rr[5] = {0.0, 0.1, 0.4, 0.8, 1.0};
#pragma unroll
                for (int k = 0; k < 5; k++) {
                    const double mj = 10.0, mn = 10.0 * rr[k];
                    const double ax = (q >= 4 ? mn : mj), ay = (q >= 4 ? mj : mn);
                    obinp |= (unsigned)whichbin((q & 1) ? ax : -ax, (q <= 1 || q >= 6) ? ay : -ay) << (6 * k);
                }
                obinp = __builtin_amdgcn_readfirstlane(obinp);
            }
#define OBIN(k) ((int)__builtin_amdgcn_ubfe(obinp, (unsigned)(6 * (k)), 6u))
            int depth = 0;
            MK_T(9);
            // cell word of candidate t = lane of the next depth, loaded while this depth finishes: the
            // next depth's candidates are known before its collectgarbage, and they stay the same
            // when that adds no block (nb == 0: the gap list is unchanged)
            uint32_t pf_w = 0;
#if MK_PFIND
            int pf_ind = 0;                     // the prefetched depth's first chunk: candidate index and gap bounds
            int2 pf_gc = make_int2(0, -1);
#endif
            bool pf_ok = false;
            int pf_T = 0;   // candidates of the prefetched depth (its ranges are in L.ga / gpre / gc)
            for (;;) {
                // ---------------- collectgarbage (sparksieve2.cpp:89-132) for the previous depth
                int nb = L.misc[1];
                if (nb > 0) pf_ok = false;
                if (PROF && nb > 0) { mst[0]++; mst[1] += (nb == 1); mst[2] += nb; mst[3] += ng; }
                if (nb > bcap + P.spill_cap) { failed = true; if (lane == 0) atomicOr(P.error, KERR_BLOCK_CAPACITY); }
                if (failed) break;
                if (nb == 1 && ng <= 64) {
                    // One block K (the common case): the sequential walk below meets every gap before the one
                    // where K is consumed with K itself, and leaves the gaps after it unchanged -- and for those
                    // gaps the same rule, applied to (gap, K) alone, also gives "unchanged" (they start past
                    // K's end).  So each gap's 0, 1 or 2 output gaps are a function of the gap and K, computed
                    // in the gap's lane, and placed by a wave prefix count.
                    const double2 kb = L.blocks[0];
                    const double kx = kb.x, ky = kb.y;
                    const bool have = lane < ng;
                    double gx = 0.0, gy = 0.0;
                    if (have) { const double2 v = L.gaps[lane]; gx = v.x; gy = v.y; }
                    double ax = gx, ay = gy, bx2 = 0.0, by2 = 0.0;
                    int nout = have ? 1 : 0;
                    if (have && !(ky < gx)) {
                        bool create = true;
                        double cx_ = gx, cy_ = gy;
                        if (kx <= cx_) { create = false; if (ky > cx_) cx_ = ky; }
                        if (ky >= cy_) { create = false; if (kx < cy_) cy_ = kx; }
                        ax = cx_;
                        ay = cy_;
                        if (cy_ <= cx_ + 1e-10) nout = 0;
                        else if (!(ky > cy_) && create) { nout = 2; ay = kx; bx2 = ky; by2 = cy_; }
                    }
                    const unsigned long long m1 = ballot(nout >= 1), m2 = ballot(nout == 2);
                    const int pos = prefix_popc(m1) + prefix_popc(m2);
                    const int no = __popcll(m1) + __popcll(m2);
                    if (no > gcap) { if (lane == 0) atomicOr(P.error, KERR_GAP_CAPACITY); failed = true; break; }
                    wave_sync();
                    if (nout >= 1) L.gaps[pos] = make_double2(ax, ay);
                    if (nout == 2) L.gaps[pos + 1] = make_double2(bx2, by2);
                    ng = no;
                    if (lane == 0) L.misc[1] = 0;
                    wave_sync();
                } else if (nb > 0 && nb <= 64 && nb <= bcap && ng <= 64) {
                    // Register path (a few blocks): lane i holds block i and lane g gap g; the
                    // dedup, the ranks and the serial merge read other lanes through v_readlane
                    // (wave-uniform indices) instead of chains of dependent LDS reads.
                    const bool valid = lane < nb;
                    double bx = 0.0, by = 0.0;
                    if (valid) { const double2 v = L.blocks[lane]; bx = v.x; by = v.y; }
                    int first = valid ? 1 : 0;
                    for (int j = 0; j < nb; j++) {
                        const double ox = readlane_d(bx, j), oy = readlane_d(by, j);
                        if (j < lane && ox == bx && oy == by) first = 0;
                    }
                    int rank = 0;
                    for (int j = 0; j < nb; j++) {
                        const int fj = __builtin_amdgcn_readlane(first, j);
                        const double ox = readlane_d(bx, j), oy = readlane_d(by, j);
                        if (fj && zone_less(ox, oy, bx, by)) rank++;
                    }
                    const int nu = __popcll(ballot(valid && first));
                    if (valid && first) L.bsorted[rank] = make_double2(bx, by);
                    double gx = 0.0, gy = 0.0;
                    if (lane < ng) { const double2 v = L.gaps[lane]; gx = v.x; gy = v.y; }
                    wave_sync();
                    double sx = 0.0, sy = 0.0;
                    if (lane < nu) { const double2 v = L.bsorted[lane]; sx = v.x; sy = v.y; }
                    // sparkSieve2::collectgarbage (sparksieve2.cpp:89-132), wave-uniform
                    int gi = 0, bi = 0, no = 0;
                    double cx_ = readlane_d(gx, 0), cy_ = readlane_d(gy, 0);
                    while (bi < nu && gi < ng) {
                        const double kx = readlane_d(sx, bi), ky = readlane_d(sy, bi);
                        if (ky < cx_) { bi++; continue; }
                        bool create = true;
                        if (kx <= cx_) { create = false; if (ky > cx_) cx_ = ky; }
                        if (ky >= cy_) { create = false; if (kx < cy_) cy_ = kx; }
                        if (cy_ <= cx_ + 1e-10) {
                            gi++;
                            if (gi < ng) { cx_ = readlane_d(gx, gi); cy_ = readlane_d(gy, gi); }
                            continue;
                        } else if (ky > cy_) {
                            if (lane == 0 && no < gcap) L.gaps2[no] = make_double2(cx_, cy_);
                            no++;
                            gi++;
                            if (gi < ng) { cx_ = readlane_d(gx, gi); cy_ = readlane_d(gy, gi); }
                            continue;
                        } else if (create) {
                            if (lane == 0 && no < gcap) L.gaps2[no] = make_double2(cx_, kx);
                            no++;
                            cx_ = ky;
                        }
                        bi++;
                    }
                    if (gi < ng) {
                        if (lane == 0 && no < gcap) L.gaps2[no] = make_double2(cx_, cy_);
                        no++;
                        // the untouched gaps gi+1 .. ng-1, in parallel from their lanes
                        if (lane > gi && lane < ng && no + (lane - gi - 1) < gcap) L.gaps2[no + (lane - gi - 1)] = make_double2(gx, gy);
                        no += ng - gi - 1;
                    }
                    if (no > gcap) { if (lane == 0) atomicOr(P.error, KERR_GAP_CAPACITY); failed = true; break; }
                    wave_sync();
                    ng = no;
                    for (int i = lane; i < ng; i += 64) L.gaps[i] = L.gaps2[i];
                    if (lane == 0) L.misc[1] = 0;
                    wave_sync();
                } else if (nb > 0) {
                    __syncthreads();   // spilled blocks written by other lanes live in HBM: drain the stores
                    // std::sort (start asc, end desc) + std::unique: first-occurrence flags, then
                    // each distinct block lands at its rank among the distinct blocks.  Blocks past
                    // the LDS capacity live in this wave's HBM spill area (rare: long walls across
                    // the sweep front); the same code reads both through get_block / set_flag.
                    for (int i = lane; i < nb; i += 64) {
                        const double2 me = get_block(i);
                        int first = 1;
                        for (int j = 0; j < i; j++) {
                            const double2 o = get_block(j);
                            if (o.x == me.x && o.y == me.y) { first = 0; break; }
                        }
                        set_flag(i, first);
                    }
                    __syncthreads();
                    int nu = 0;
                    for (int i = lane; i < nb; i += 64) {
                        if (!get_flag(i)) continue;
                        const double2 me = get_block(i);
                        int rank = 0;
                        for (int j = 0; j < nb; j++) {
                            const double2 o = get_block(j);
                            if (get_flag(j) && zone_less(o.x, o.y, me.x, me.y)) rank++;
                        }
                        put_sorted(rank, me);
                    }
                    for (int base = 0; base < nb; base += 64) nu += __popcll(ballot(base + lane < nb && get_flag(base + lane)));
                    __syncthreads();
                    // sequential merge on lane 0: gaps -> gaps2
                    if (lane == 0) {
                        int gi = 0, bi = 0, no = 0;
                        bool over = false;
                        double2 cur = (ng > 0) ? L.gaps[0] : make_double2(0, 0);
                        while (bi < nu && gi < ng) {
                            const double2 bk = get_sorted(bi);
                            if (bk.y < cur.x) { bi++; continue; }
                            bool create = true;
                            if (bk.x <= cur.x) { create = false; if (bk.y > cur.x) cur.x = bk.y; }
                            if (bk.y >= cur.y) { create = false; if (bk.x < cur.y) cur.y = bk.x; }
                            if (cur.y <= cur.x + 1e-10) {
                                gi++;
                                if (gi < ng) cur = L.gaps[gi];
                                continue;
                            } else if (bk.y > cur.y) {
                                if (no < gcap) L.gaps2[no] = cur; else over = true;
                                no++;
                                gi++;
                                if (gi < ng) cur = L.gaps[gi];
                                continue;
                            } else if (create) {
                                if (no < gcap) L.gaps2[no] = make_double2(cur.x, bk.x); else over = true;
                                no++;
                                cur.x = bk.y;
                            }
                            bi++;
                        }
                        if (gi < ng) {
                            if (no < gcap) L.gaps2[no] = cur; else over = true;
                            no++;
                            for (int g = gi + 1; g < ng; g++) {
                                if (no < gcap) L.gaps2[no] = L.gaps[g]; else over = true;
                                no++;
                            }
                        }
                        if (over) { atomicOr(P.error, KERR_GAP_CAPACITY); no = -1; }
                        L.misc[0] = no;
                    }
                    __syncthreads();
                    ng = L.misc[0];
                    if (ng < 0) { failed = true; break; }
                    for (int i = lane; i < ng; i += 64) L.gaps[i] = L.gaps2[i];
                    if (lane == 0) L.misc[1] = 0;
                    __syncthreads();
                }
                MK_T(0);
                // loop condition: sieve.hasGaps() (pointdata.cpp:1454)
                if (ng == 0) break;
                depth++;
                if (COUNT || PROF) nsteps++;
                // ---------------- sieve2 for this depth (pointdata.cpp:1512-1565)
                // per-gap visit ranges with the monotone firstind rule
                int carryF = 0, carryT = 0;
                if (ng <= 8 && pf_ok) {
                    // the previous depth's prefetch already laid out this depth's ranges (same gap list)
                    carryT = pf_T;
                } else if (ng <= 8) {
                    // few gaps (the common case): a wave-uniform loop over the gaps in order -- no
                    // cross-lane scans.  F = the largest b of the earlier visited gaps (at least 0).
                    int F = 0, T = 0;
                    for (int g = 0; g < ng; g++) {
                        const double2 z = L.gaps[g];
                        const int lo = (int)ceil(z.x * (depth - 0.5) - 0.5);
                        const int hi = (int)floor(z.y * (depth + 0.5) + 0.5);
                        const int b = min(hi, depth);
                        const int a = max(lo, F);
                        const int c = (b >= a) ? (b - a + 1) : 0;
                        if (lane == 0) {
                            L.ga[g] = a;
                            L.gpre[g] = T;
                            L.gc[g] = make_int2((int)ceil(z.x * depth), (int)floor(z.y * depth));
                        }
                        T += c;
                        if (b >= lo) F = max(F, b);
                    }
                    carryT = T;
                }
                for (int base = 0; base < ng && ng > 8; base += 64) {
                    int g = base + lane;
                    int lo = 0, b = -1;
                    bool vis = false;
                    if (g < ng) {
                        double2 z = L.gaps[g];
                        lo = (int)ceil(z.x * (depth - 0.5) - 0.5);
                        int hi = (int)floor(z.y * (depth + 0.5) + 0.5);
                        b = min(hi, depth);
                        vis = (b >= lo);
                        L.gc[g] = make_int2((int)ceil(z.x * depth), (int)floor(z.y * depth));
                    }
                    int bp = vis ? b : INT_MIN;
                    int incl = wave_incl_max(bp);
                    int excl = __shfl_up(incl, 1);
                    if (lane == 0) excl = INT_MIN;
                    int F = max(carryF, max(excl, 0));
                    int a = max(lo, F);
                    int c = (g < ng && b >= a) ? (b - a + 1) : 0;
                    int ci = wave_incl_sum(c);
                    if (g < ng) { L.ga[g] = a; L.gpre[g] = carryT + ci - c; }
                    carryT += __shfl(ci, 63);
                    carryF = max(carryF, __shfl(incl, 63));
                }
                if (lane == 0) L.gpre[ng] = carryT;
                wave_sync();
                const int T = carryT;
                examined += (unsigned long long)T;
                MK_T(1);
                bool hasgaps = false;
                int lmin = INT_MAX;   // smallest clean distance of this lane's candidates (span certificate)
                int gcur = 0; // per-lane gap pointer (t increases monotonically)
                for (int t0 = 0; t0 < T; t0 += 64) {
                    if (COUNT || PROF) nchunks++;
                    int t = t0 + lane;
                    bool valid = t < T;
                    int ind = 0, hx = 0, hy = 0;
                    int2 gcr = make_int2(0, -1);
                    bool ingrid = false, add = false;
                    uint32_t w = 0;
                    if (valid) {
#if MK_PFIND
                        if (pf_ok && t0 == 0) {   // the prefetch laid this chunk out already
                            ind = pf_ind;
                            gcr = pf_gc;
                        } else
#endif
                        {
                            while (L.gpre[gcur + 1] <= t) gcur++;
                            ind = L.ga[gcur] + (t - L.gpre[gcur]);
                            gcr = L.gc[gcur];
                        }
                        octant_cell(q, cx, cy, depth, ind, hx, hy);
                        ingrid = (hx >= 0 && hx < P.cols && hy >= 0 && hy < P.rows);
                    }
                    int nlb = 0, offb = 0;
                    if (ingrid) {
                        const int hc = hx * P.rows + hy;
                        w = (pf_ok && t0 == 0) ? pf_w : P.cellw[hc];
                        const int nl = cell_nseg(w), off = cell_seg_off(w);
                        // (double)ind >= start*depth && (double)ind <= end*depth, on the integer
                        // bounds of the two FP64 products (computed once per gap and depth)
                        const bool centregap = ind >= gcr.x && ind <= gcr.y;
                        if (centregap && cell_filled(w) &&
                            (ind != 0 || q == 0 || q == 1 || q == 5 || q == 6) && (ind != depth || q < 4)) {
                            // sparkSieve2::testblock (sparksieve2.cpp:45-63)
                            const double px = P.blx + sp * 1.0 * (double)hx, py = P.bly + sp * 1.0 * (double)hy;
                            bool blocked = false;
                            if (hasmax || nl > 0) {
                                Seg ray = make_seg(Vec2{c0x, c0y}, Vec2{px, py});
                                if (hasmax && ray.length() > P.maxdist) blocked = true;
                                const double tol = sp * 1e-10;
                                for (int k = 0; k < nl && !blocked; k++) {
                                    const double* sg = P.segs + 4 * (size_t)(off + k);
                                    Seg s = make_seg(Vec2{sg[0], sg[1]}, Vec2{sg[2], sg[3]});
                                    if (rects_touch(ray.r, s.r, tol) && segs_cross(ray, s, tol)) blocked = true;
                                }
                            }
                            add = !blocked;
                        }
                        // sparkSieve2::block for every in-grid candidate (sparksieve2.cpp:67-87)
                        for (int k = 0; k < nl; k++) {
                            const double* sg = P.segs + 4 * (size_t)(off + k);
                            double ta = tanify(c0x, c0y, sg[0], sg[1], q), tb = tanify(c0x, c0y, sg[2], sg[3], q);
                            const int slot = atomicAdd(&L.misc[1], 1);
                            put_block(slot, (ta < tb) ? make_double2(ta - 1e-10, tb + 1e-10) : make_double2(tb - 1e-10, ta + 1e-10));
                        }
                    }
                    if (valid) lmin = min(lmin, ingrid ? cell_span_dist(w) : 0);
                    hasgaps |= (ballot(ingrid) != 0ull);
                    MK_T(2);
                    // ---- visible cells: bins, moments (reference order), run tracking
                    unsigned long long am = ballot(add);
                    if (am) {
                        int bin = -1;
                        double this_dist = 0.0;
                        // whichbin(depixelate(c) - centre) (pointdata.h:432-520) decided on the exact ratio
                        // ind/depth: 0 and 1 are the axis / diagonal; tan15 and tan30 are irrational, so a float
                        // test with a 1e-6 margin decides every cell the reference's FP64 ratio (error ~1e-15)
                        // decides; cells inside the margin take the FP64 path
                        {
                            const float fd = (float)depth, fi = (float)ind, mg = 1e-6f * fd;
                            const float e15 = fi - 0.267949192f * fd, e30 = fi - 0.577350269f * fd;
                            int k = 1 + (e15 >= 0.0f) + (e30 >= 0.0f);
                            k = (ind == depth) ? 4 : k;
                            k = (ind == 0) ? 0 : k;
                            bin = OBIN(k);
                            const bool amb = add & (ind != 0) & (ind != depth) & ((fabsf(e15) < mg) | (fabsf(e30) < mg));
                            if (ballot(amb) != 0ull) {
                                if (amb) {
                                    const double px = P.blx + sp * 1.0 * (double)hx, py = P.bly + sp * 1.0 * (double)hy;
                                    bin = whichbin(px - c0x, py - c0y);
                                }
                            }
                        }
                        // dx^2 + dy^2 (exact): the far distance (:1489) is the float of the bin's largest one (the
                        // dists grow with it, and (float) rounding keeps the order)
                        const unsigned n2 = (unsigned)(depth * depth) + __umul24((unsigned)ind, (unsigned)ind);
                        if (add) {
                            atomicAdd(&L.binc[bin], 1u);
                            atomicMax(&L.bfar[bin], n2);
                        }
                        MK_T(3);
                        if (exact) {
                            // serial sums in lane order = reference addlist order
                            // (the lane index is wave-uniform: v_readlane into SGPRs keeps the serial
                            // chain on two dependent FP64 adds per cell instead of an LDS round trip)
                            if (add) this_dist = sqrt((double)n2) * sp;   // sqrt(dx*dx + dy*dy) * spacing
                            const int d_lo = __double2loint(this_dist), d_hi = __double2hiint(this_dist);
                            unsigned long long mm = am;
                            while (mm) {
                                const int l = __ffsll((long long)mm) - 1;
                                const double v = __hiloint2double(__builtin_amdgcn_readlane(d_hi, l),
                                                                  __builtin_amdgcn_readlane(d_lo, l));
                                tsum += v;
                                tsum2 += v * v;
                                mm &= mm - 1;
                            }
                        } else if (add) {
                            s1 += sqrt_nr((double)n2);
                            s2n += n2;
                            mcnt++;
                        }
                        MK_T(4);
                        nsize += __popcll(am);
                        // run tracking
                        bool emit = false;
                        unsigned long long rec = 0;
                        if (add) {
                            if (ind == depth && q < 4) { // diagonal bin: single span (ngraph.cpp:243-258)
                                if (bin != q_diag) atomicOr(P.error, KERR_BIN_MISMATCH);
                            } else {
                                int slot;
                                if (ind == 0) { slot = 3; if (bin != q_axis) atomicOr(P.error, KERR_BIN_MISMATCH); }
                                else { slot = bin - q_sector; if (slot < 0 || slot > 2) { atomicOr(P.error, KERR_BIN_MISMATCH); slot = 0; } }
                                uint32_t o = ld_open(ind);
                                int oslot = (o >> 1) & 3, os = (o >> 3) & 0x3fff, ol = (o >> 17) & 0x3fff;
                                if ((o & 1u) && oslot == slot && ol == depth - 1) {
                                    st_open(ind, pack_open(slot, os, depth) | (o & MK_OPEN_ADJ));
                                } else {
                                    // a run that ends where the row's next run starts (a bin boundary, not a
                                    // gap): the two runs' facing ends need no symmetry range adds
                                    const bool adj = (o & 1u) && ol == depth - 1;
                                    if (o & 1u) {   // the rank within (slot, row) is set after the octant
                                        emit = true;
                                        rec = pack_emit(oslot, ind, os, ol, 0) | ((unsigned long long)(o >> 31) << MK_REC_SHALLOW) |
                                              ((unsigned long long)adj << MK_REC_DEEP);
                                    }
                                    st_open(ind, pack_open(slot, depth, depth) | (adj ? MK_OPEN_ADJ : 0u));
                                }
                            }
                        }
                        // the diagonal cell (at most one per depth) -- wave-uniform bookkeeping
                        unsigned long long dm = ballot(add && ind == depth && q < 4);
                        if (dm) {
                            if (diag_n == 0) diag_min = depth;
                            diag_max = depth;
                            diag_n++;
                        }
                        unsigned long long em = ballot(emit);
                        if (em) {
                            int pos = nA + prefix_popc(em);
                            if (emit) {
                                if (pos < P.capA) stA[pos] = rec;
                            }
                            nA += __popcll(em);
                        }
                    }
                    MK_T(5);
                }
                if (nA > P.capA) { failed = true; if (lane == 0) atomicOr(P.error, KERR_STAGE_CAPACITY); }
                if (!hasgaps) break;      // sieve2 returned false (pointdata.cpp:1458)
                dq = depth;
                // ---------------- occluder-free span: depths depth+1 .. depth+k in one pass (span.hpp)
                // Certificate: this depth added no block, and every cell it visited has clean distance >= k + 2.
                // The rows a gap visits at depth + j lie within j + 1 rows of the rows it visits here (lo and
                // firstind never fall, hi rises by at most j + 1), so every cell visited at depths depth+1 ..
                // depth+k is within Chebyshev distance k + 1 of a cell visited here: FILLED, in the grid, without
                // an occluder piece.  Those depths add no block (the gap list stays), every visited cell in a
                // gap's centre is visible, and a row's visible depths are an interval per gap.  The rows are
                // spread over the lanes; a row's runs, bin counts and far distances come per (gap, ratio class)
                // interval, only the first moment's square roots per cell.
                // (expect false: the register allocator weighs the span's loops below the candidate loop's)
                if (__builtin_expect(spans && !failed && L.misc[1] == 0 && ballot(lmin < span_min + 2) == 0ull, 0)) {
                    int mind = lmin;
#if MK_WFRED
                    mind = __ockl_wfred_min_i32(mind);
#else
                    for (int off = 32; off >= 1; off >>= 1) mind = min(mind, __shfl_xor(mind, off));
#endif
                    const int d0 = depth + 1, d1 = depth + (mind - 2);
                    if (far_rows) __syncthreads(); else wave_sync();   // this depth's open-row stores
                    SpanOct so;
                    so.q = q; so.cx = cx; so.cy = cy; so.blx = P.blx; so.bly = P.bly; so.sp = sp; so.c0x = c0x; so.c0y = c0y;
                    so.obinp = obinp;
                    const bool axis_row = (q == 0 || q == 1 || q == 5 || q == 6);
                    // reciprocals of the gap ends in L.gaps2 (free outside collectgarbage): row estimates, which the
                    // exact predicates then settle
                    for (int g = lane; g < ng; g += 64) {
                        const double2 z = L.gaps[g];
#if MK_SPAN_RCP
                        L.gaps2[g] = make_double2(__builtin_amdgcn_rcp(z.x), __builtin_amdgcn_rcp(z.y));
#else
                        L.gaps2[g] = make_double2(1.0 / z.x, 1.0 / z.y);
#endif
                    }
                    wave_sync();
                    const int R0 = max(0, gap_cl(L.gaps[0].x, d0)), R1 = min(d1, gap_ch(L.gaps[ng - 1].y, d1));
                    int nsp = 0;   // this lane's visible cells in the span
                    for (int rb = R0; rb <= R1; rb += 64) {
                        if (COUNT || PROF) nchunks++;
                        const int ind = rb + lane;
                        const bool live = ind <= R1;
                        // last depths of ratio classes 3 and 2 (span.hpp class_last), settled exactly only when
                        // they fall near the span (ind / tan is within 1e-11 of the product below)
                        int t3 = ind, t2 = ind;
                        if (live && ind > 0) {
                            const double x3 = (double)ind * 1.7320508075688772, x2 = (double)ind * 3.7320508075688776;
                            t3 = (x3 + 3.0 < (double)d0) ? d0 - 1 : (x3 - 3.0 > (double)d1) ? d1
                                                                  : class_last(so, ind, 3, 0.5773502691896257);
                            t2 = (x2 + 3.0 < (double)d0) ? d0 - 1 : (x2 - 3.0 > (double)d1) ? d1
                                                                  : class_last(so, ind, 2, 0.2679491924311227);
                            t3 = max(t3, ind);
                            t2 = max(t2, t3);
                        }
                        uint32_t o = live ? ld_open(ind) : 0u;
                        bool diag = false;
                        if (PROF) spst[3]++;
                        MK_T(11);
                        for (int g = ng - 1; g >= 0; g--) {   // later gaps first: the row's depths in order
                            const double2 z = L.gaps[g], iz = L.gaps2[g];
                            const double gs_ = z.x, ge_ = z.y;
#if MK_SPAN_GSKIP
                            // rows below cl(s, d0) or above ch(e, d1) see no depth of the span in this gap
                            if (ballot(live && ind >= gap_cl(gs_, d0) && ind <= gap_ch(ge_, d1)) == 0ull) continue;
#endif
                            int p = 1, r = 0;
                            if (live) {
                                // first d with ch(e, d) >= ind; last d with cl(s, d) <= ind and b(e_prev, d) <= ind
                                int a = (ind == 0) ? d0 : clamp_est(ceil((double)ind * iz.y), d0, d1 + 1);
                                while (a > d0 && gap_ch(ge_, a - 1) >= ind) a--;
                                while (a <= d1 && gap_ch(ge_, a) < ind) a++;
                                int c = (gs_ > 0.0) ? clamp_est(floor((double)ind * iz.x), d0 - 1, d1) : d1;
                                while (c < d1 && gap_cl(gs_, c + 1) <= ind) c++;
                                while (c >= d0 && gap_cl(gs_, c) > ind) c--;
                                if (g > 0) {
                                    const double gp_ = L.gaps[g - 1].y;
                                    int f = clamp_est(floor(((double)ind + 0.5) * L.gaps2[g - 1].y - 0.5), d0 - 1, d1);
                                    const int m = min(ind, d1);
                                    if (f < m) f = m;
                                    while (f < d1 && gap_b(gp_, f + 1) <= ind) f++;
                                    while (f >= d0 && gap_b(gp_, f) > ind) f--;
                                    c = min(c, f);
                                }
                                p = a;
                                r = c;
                                if (ind == 0 && !axis_row) r = p - 1;      // (ind != 0 || q in {0,1,5,6})
                                if (q >= 4 && p <= ind) p = ind + 1;       // (ind != depth || q < 4)
                            }
                            if (p <= r) {
                                // two independent chains (any summation order is within the certificate's bound)
                                double sa = 0.0, sb = 0.0;
                                const unsigned i2 = (unsigned)(ind * ind);
                                int d = p;
                                for (; d + 1 <= r; d += 2) {
                                    sa += sqrt_nr((double)((unsigned)(d * d) + i2));
                                    sb += sqrt_nr((double)((unsigned)((d + 1) * (d + 1)) + i2));
                                }
                                if (d <= r) sa += sqrt_nr((double)((unsigned)(d * d) + i2));
                                s1 += sa + sb;
                                const unsigned long long ur = (unsigned long long)r, up = (unsigned long long)(p - 1);
                                s2n += (ur * (ur + 1) * (2 * ur + 1) - up * (up + 1) * (2 * up + 1)) / 6 +
                                       (unsigned long long)(r - p + 1) * (unsigned long long)(ind * ind);
                                mcnt += r - p + 1;
                                nsp += r - p + 1;
                            }
                            // pieces in depth order: the diagonal cell, ratio classes 3, 2, 1 (row 0: the axis, class 0);
                            // only the classes some lane has
                            const bool has = p <= r;
                            if (PROF) { spst[4]++; spst[5] += (ballot(has) == 0ull); }
                            MK_T(12);
                            const int chi = (ind == 0) ? 0 : (ind >= p && ind <= r) ? 4 : (p <= t3) ? 3 : (p <= t2) ? 2 : 1;
                            const int clo = (ind == 0) ? 0 : (r <= t3) ? 3 : (r <= t2) ? 2 : 1;
#if MK_SPAN_CB
                            // the classes in some lane's [clo, chi], highest first (the others have no piece anywhere)
                            unsigned cset = 0;
#pragma unroll
                            for (int c5 = 0; c5 < 5; c5++) cset |= (ballot(has && clo <= c5 && c5 <= chi) != 0ull) ? (1u << c5) : 0u;
                            for (; cset; cset &= ~(1u << (31 - __clz((int)cset)))) {
                                const int cc = 31 - __clz((int)cset);
#else
                            int cmax = wave_incl_max_all(has ? chi : -1), cmin = -wave_incl_max_all(has ? -clo : -5);
                            for (int cc = cmax; cc >= cmin; cc--) {
#endif
                                int a = 1, b = 0;
                                if (ind == 0) { if (cc == 0) { a = p; b = r; } }
                                else if (cc == 4) { a = max(p, ind); b = min(r, ind); }
                                else if (cc == 3) { a = max(p, ind + 1); b = min(r, t3); }
                                else if (cc == 2) { a = max(p, t3 + 1); b = min(r, t2); }
                                else if (cc == 1) { a = max(p, t2 + 1); b = r; }
                                bool emit = false;
                                unsigned long long rec = 0;
                                if (live && a <= b) {
                                    const int bin = OBIN(cc);
                                    atomicAdd(&L.binc[bin], (unsigned)(b - a + 1));
                                    atomicMax(&L.bfar[bin], (unsigned)(b * b + ind * ind));
                                    if (cc == 4) {
                                        diag = true;
                                    } else {   // the per-cell run tracking below, for the cells a..b at once
                                        const int slot = (cc == 0) ? 3 : bin - q_sector;
                                        const int oslot = (o >> 1) & 3, os = (o >> 3) & 0x3fff, ol = (o >> 17) & 0x3fff;
                                        if ((o & 1u) && oslot == slot && ol == a - 1) {
                                            o = pack_open(slot, os, b) | (o & MK_OPEN_ADJ);
                                        } else {
                                            const bool adj = (o & 1u) && ol == a - 1;
                                            if (o & 1u) {
                                                emit = true;
                                                rec = pack_emit(oslot, ind, os, ol, 0) | ((unsigned long long)(o >> 31) << MK_REC_SHALLOW) |
                                                      ((unsigned long long)adj << MK_REC_DEEP);
                                            }
                                            o = pack_open(slot, a, b) | (adj ? MK_OPEN_ADJ : 0u);
                                        }
                                    }
                                }
                                const unsigned long long em = ballot(emit);
                                if (em) {
                                    const int pos = nA + prefix_popc(em);
                                    if (emit && pos < P.capA) stA[pos] = rec;
                                    nA += __popcll(em);
                                }
                            }
                            MK_T(13);
                        }
                        if (live) st_open(ind, o);
                        const unsigned long long dm = ballot(diag);   // diagonal cells: rows ascending = depths ascending
                        if (dm) {
                            if (diag_n == 0) diag_min = rb + (__ffsll((long long)dm) - 1);
                            diag_max = rb + 63 - __clzll((long long)dm);
                            diag_n += __popcll(dm);
                        }
                    }
                    // cells examined (stats[0]): the visit ranges of every span depth, one depth a lane
                    unsigned long long exs = 0;
                    for (int db = d0; db <= d1; db += 64) {
                        const int d = db + lane;
                        int F = 0, T = 0;
                        for (int g = 0; g < ng; g++) {
                            const double2 z = L.gaps[g];
                            const int lo = gap_lo(z.x, d), b = min(gap_hi(z.y, d), d), a = max(lo, F);
                            T += (b >= a) ? (b - a + 1) : 0;
                            if (b >= lo) F = max(F, b);
                        }
                        if (d <= d1) exs += (unsigned long long)T;
                    }
#if MK_SPAN_LSUM
                    examined_l += exs;
                    nsize_l += nsp;
                    if (PROF) {
                        for (int off = 32; off >= 1; off >>= 1) nsp += __shfl_xor(nsp, off);
                        spst[0]++; spst[1] += (unsigned long long)(d1 - d0 + 1); spst[2] += (unsigned long long)__shfl(nsp, 0);
                    }
#else
                    for (int off = 32; off >= 1; off >>= 1) {
                        exs += __shfl_xor(exs, off);
                        nsp += __shfl_xor(nsp, off);
                    }
                    examined += __shfl(exs, 0);
                    nsize += __shfl(nsp, 0);
                    if (PROF) { spst[0]++; spst[1] += (unsigned long long)(d1 - d0 + 1); spst[2] += (unsigned long long)__shfl(nsp, 0); }
#endif
                    if (COUNT || PROF) nsteps++;
                    depth = d1;
                    dq = depth;
                    if (nA > P.capA) { failed = true; if (lane == 0) atomicOr(P.error, KERR_STAGE_CAPACITY); }
                    // the open-row stores (LDS; scratch rows past MK_OPEN_LDS) before the next depth reads them
                    if (far_rows) __syncthreads(); else wave_sync();
                    MK_T(10);
                }
                // prefetch: candidate t = lane of depth + 1 under the current gap list (few-gap case)
                pf_ok = false;
                // (a depth that added blocks changes the gap list: its next depth recomputes the ranges and
                // reloads its cells, so nothing is prefetched for it)
                if (ng <= 8 && !failed && L.misc[1] == 0) {
                    const int d1 = depth + 1;
                    int F1 = 0, T1 = 0, pind = -1;
                    for (int g = 0; g < ng; g++) {
                        const double2 z = L.gaps[g];
                        const int lo = (int)ceil(z.x * (d1 - 0.5) - 0.5);
                        const int hi = (int)floor(z.y * (d1 + 0.5) + 0.5);
                        const int b = min(hi, d1);
                        const int a = max(lo, F1);
                        const int c = (b >= a) ? (b - a + 1) : 0;
                        const int2 gcg = make_int2((int)ceil(z.x * d1), (int)floor(z.y * d1));
                        if (lane >= T1 && lane < T1 + c) {
                            pind = a + (lane - T1);
#if MK_PFIND
                            pf_gc = gcg;
#endif
                        }
                        if (lane == 0) {   // depth d1's visit ranges, reused if no block changes the gaps
                            L.ga[g] = a;
                            L.gpre[g] = T1;
                            L.gc[g] = gcg;
                        }
                        T1 += c;
                        if (b >= lo) F1 = max(F1, b);
                    }
                    pf_T = T1;
#if MK_PFIND
                    pf_ind = pind;
#endif
                    if (pind >= 0) {
                        int px, py;
                        octant_cell(q, cx, cy, d1, pind, px, py);
                        if (px >= 0 && px < P.cols && py >= 0 && py < P.rows) pf_w = P.cellw[px * P.rows + py];
                    }
                    pf_ok = true;
                }
                MK_T(8);
                // rows past MK_OPEN_LDS live in scratch memory: order this depth's stores before the next
                // depth's loads of the same rows (other lanes); only sight lines past 1024 cells get here
                if (depth >= MK_OPEN_LDS) __syncthreads();
                wave_sync();
            }
            if (failed) break;
            // ---------------- flush open rows, then place this octant's runs canonically
            __syncthreads();
            for (int base = 0; base <= dq; base += 64) {
                int ind = base + lane;
                bool emit = false;
                unsigned long long rec = 0;
                if (ind <= dq) {
                    uint32_t o = ld_open(ind);
                    if (o & 1u) {
                        int oslot = (o >> 1) & 3, os = (o >> 3) & 0x3fff, ol = (o >> 17) & 0x3fff;
                        emit = true;
                        rec = pack_emit(oslot, ind, os, ol, 0) | ((unsigned long long)(o >> 31) << MK_REC_SHALLOW);
                    }
                    st_open(ind, 0u);
                }
                unsigned long long em = ballot(emit);
                if (em) {
                    int pos = nA + prefix_popc(em);
                    if (emit && pos < P.capA) stA[pos] = rec;
                    nA += __popcll(em);
                }
            }
            if (nA > P.capA) { failed = true; if (lane == 0) atomicOr(P.error, KERR_STAGE_CAPACITY); break; }
            __syncthreads();
            // ranks within (slot, row): the runs of one row and slot are staged in depth order, so a
            // record's rank is the number of earlier records with its key (earlier chunks: the running
            // count in rcnt; this chunk: earlier lanes with the same key)
            for (int base = 0; base < nA; base += 64) {
                const int i = base + lane;
                unsigned long long rec = 0;
                int key = -1;
                if (i < nA) {
                    rec = stA[i];
                    const int slot = (int)(rec & 3ull), ind = (int)((rec >> 2) & 0x3fff);
                    key = (slot == 3) ? AX : slot * (D + 1) + ind;
                }
                int r = 0;
                bool last = true;
                const int n = min(64, nA - base);
                for (int j = 0; j < n; j++) {
                    const int kj = __builtin_amdgcn_readlane(key, j);
                    if (kj == key) {
                        if (j < lane) r++;
                        else if (j > lane) last = false;
                    }
                }
                if (key >= 0) {
                    const uint32_t k = ld_l2(&rcnt[key]) + (uint32_t)r;
                    stA[i] = rec | ((unsigned long long)k << 44);
                    if (last) st_l2(&rcnt[key], k + 1);
                }
                __syncthreads();   // the next chunk reads these counters (other lanes, same wave)
            }
            __syncthreads();
            // exclusive prefix over (slot, canonical row) -> pref[]
            const int R1 = dq + 1;
            const int nkeys = 3 * R1;
            const int rasc = c_row_asc[q], dasc = c_d_asc[q];
            int carry = 0;
            for (int base = 0; base < nkeys; base += 64) {
                int key = base + lane;
                int c = 0;
                if (key < nkeys) {
                    int slot = key / R1, r = key % R1;
                    int ind = rasc ? r : (dq - r);
                    c = (int)ld_l2(&rcnt[slot * (D + 1) + ind]);
                }
                int ci = wave_incl_sum(c);
                if (key < nkeys) pref[key] = carry + ci - c;
                carry += __shfl(ci, 63);
            }
            const int nsector = carry;
            const int axis_runs = (int)ld_l2(&rcnt[AX]);
            if (lane == 0) pref[nkeys] = carry;
            // per-bin run counts for the sectors
            {
                int s0 = 0, s1 = 0;
                // slot boundaries in key space are multiples of R1
                __syncthreads();
                s0 = pref[R1];
                s1 = pref[2 * R1];
                if (lane == 0) {
                    L.bnr[q_sector + 0] += s0;
                    L.bnr[q_sector + 1] += s1 - s0;
                    L.bnr[q_sector + 2] += nsector - s1;
                    if (q_axis >= 0) L.bnr[q_axis] += axis_runs;
                    if (q_diag >= 0) L.bnr[q_diag] += (diag_n > 0) ? 1 : 0;
                }
            }
            const int diag_runs = (diag_n > 0) ? 1 : 0;
            int low_n = 0;
            if (c_axis_low[q]) low_n = axis_runs;
            if (c_diag_low[q]) low_n = diag_runs;
            const int seg_len = low_n + nsector + (c_axis_low[q] ? 0 : (q_axis >= 0 ? axis_runs : 0)) +
                                (c_diag_low[q] ? 0 : diag_runs);
            if (bpos + seg_len > P.capB) { failed = true; if (lane == 0) atomicOr(P.error, KERR_STAGE_CAPACITY); break; }
            Run* seg = stB + bpos;
            const int high_base = low_n + nsector;
            __syncthreads();
            for (int i = lane; i < nA; i += 64) {
                unsigned long long rec = stA[i];
                int slot = (int)(rec & 3ull), ind = (int)((rec >> 2) & 0x3fff), ds = (int)((rec >> 16) & 0x3fff);
                int de = (int)((rec >> 30) & 0x3fff), k = (int)((rec >> 44) & 0x3fff);
                int pos;
                if (slot == 3) {
                    int base = c_axis_low[q] ? 0 : high_base;
                    pos = base + (dasc ? k : (axis_runs - 1 - k));
                } else {
                    int r = rasc ? ind : (dq - ind);
                    int key = slot * R1 + r;
                    pos = low_n + (dasc ? (int)pref[key] + k : (int)pref[key + 1] - 1 - k);
                }
                Run ru = make_run(q, cx, cy, ind, ds, de);
                if (symflags) {   // the adjacency bits, from depth order (shallow / deep end) to start / end
                    const bool sh = (rec >> MK_REC_SHALLOW) & 1ull, dp = (rec >> MK_REC_DEEP) & 1ull;
                    const bool inc = (q < 4) ? (q & 1) != 0 : (q >= 6);   // coordinate grows with depth
                    if (inc ? sh : dp) ru.x0 |= MK_RUN_FLAG;
                    if (inc ? dp : sh) ru.x1 |= MK_RUN_FLAG;
                }
                seg[pos] = ru;
            }
            if (diag_runs && lane == 0) {
                // Bin::make diagonal: first pushed pixel, replaced by the last one if it lies left/right
                int fx, fy, lx, ly;
                octant_cell(q, cx, cy, diag_min, diag_min, fx, fy);
                octant_cell(q, cx, cy, diag_max, diag_max, lx, ly);
                Run r;
                r.x0 = fx; r.y0 = fy; r.x1 = fx; r.y1 = fy;
                if (lx < r.x0) { r.x0 = lx; r.y0 = ly; }
                if (lx > r.x1) { r.x1 = lx; r.y1 = ly; }
                int pos = c_diag_low[q] ? 0 : high_base;
                seg[pos] = r;
            }
            // reset the per-row counters used by this octant
            __syncthreads();
            for (int i = lane; i < AX; i += 64)
                if (i % (D + 1) <= dq) st_l2(&rcnt[i], 0u);
            if (lane == 0) { st_l2(&rcnt[AX], 0u); L.misc[16 + q] = bpos; L.misc[24 + q] = seg_len; }
            bpos += seg_len;
            __syncthreads();
            MK_T(6);
        }
#if MK_SPAN_LSUM
        for (int off = 32; off >= 1; off >>= 1) {
            nsize_l += __shfl_xor(nsize_l, off);
            examined_l += __shfl_xor(examined_l, off);
        }
        nsize += __shfl(nsize_l, 0);
        examined += __shfl(examined_l, 0);
#endif
        float m1f = 0.0f, m2f = 0.0f;
        if (!failed) {
            if (exact) {
                m1f = (float)tsum;
                m2f = (float)tsum2;
            } else {
                int mmax = mcnt;
                for (int off = 32; off >= 1; off >>= 1) {
                    s1 += __shfl_xor(s1, off);
                    s2 += __shfl_xor(s2, off);
                    s2n += __shfl_xor(s2n, off);
                    mmax = max(mmax, __shfl_xor(mmax, off));
                }
                // lanes reduce in different orders: take lane 0's sums
                s1 = __shfl(s1, 0); s2 = __shfl(s2, 0);
                // The reference's serial chains (pointdata.cpp:1490-1495) are within gamma_(n-1) of the exact sums
                // of their terms, and those within 2u (dist) and 5u (dist^2) of sp*sqrt(n_i) and sp^2*n_i.  Ours:
                // the lanes' sums of approximate roots (each within sqrt_err) reduced by a 6-level butterfly
                // (gamma_(m+6)) times sp; the exact integer sum times sp^2 (3u).  E bounds |ours - reference| with
                // a factor 2 to spare.
                const double S1 = s1 * sp, S2 = (double)s2n * (sp * sp);
                const double u = 0x1p-53;
                const double g1 = (double)nsize * u / (1.0 - (double)nsize * u);
                const double g2 = (double)(mmax + 7) * u / (1.0 - (double)(mmax + 7) * u);
                const bool ok1 = certified_float_e(S1, 2.0 * (g1 + g2 + P.sqrt_err) * S1 + S1 * 0x1p-49, &m1f);
                const bool ok2 = certified_float_e(S2, 2.0 * g1 * S2 + S2 * 0x1p-48, &m2f);
                if (!(ok1 && ok2)) { failed = true; certfail = true; }
            }
        }
        if (failed) {
            if (lane == 0) P.fail_list[atomicAdd(P.fail_count, 1)] = node | (certfail ? 0 : MK_CAPACITY_TAG);
            // leave the wave in a clean LDS state and drop this source
            for (int i = lane; i < D + 4; i += 64) st_open(i, 0u);
            for (int i = lane; i <= AX; i += 64) st_l2(&rcnt[i], 0u);
            __syncthreads();
            continue;
        }
        // ---------------- publish: reserve pool space, copy segments in bin order 0..31
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(P.pool_cursor, (unsigned long long)bpos);
        base = __shfl(base, 0);
        const int64_t k = node - P.node_begin;
        if ((int64_t)(base + bpos) > P.pool_capacity) {
            if (lane == 0) atomicOr(P.error, KERR_POOL_CAPACITY);
            P.node_run_start[k] = -1;
        } else {
            int64_t dst = (int64_t)base;
            const bool sym = P.sym_diff != nullptr;
            const unsigned long long su = sym ? cell_weight((unsigned long long)cell) : 0ull;
            unsigned long long ho = 0ull;   // 64-bit wrap-around: the order of the terms does not matter
            for (int si = 0; si < 8; si++) {
                int q = c_seg_order[si];
                const Run* src = stB + L.misc[16 + q];
                const int len = L.misc[24 + q];
                for (int i = lane; i < len; i += 64) {
                    Run r = src[i];
                    bool skip0 = false, skip1 = false;
                    if (symflags) {
                        skip0 = (r.x0 & MK_RUN_FLAG) != 0;
                        skip1 = (r.x1 & MK_RUN_FLAG) != 0;
                        r.x0 &= ~MK_RUN_FLAG;
                        r.x1 &= ~MK_RUN_FLAG;
                    }
                    P.pool[dst + i] = r;
                    if (sym) ho += sym_run_scatter_q(r, q, skip0, skip1, su, P.cols, P.rows, P.sym_prefix, P.sym_diff);
                }
                dst += len;
            }
            if (sym) {
                for (int off = 32; off >= 1; off >>= 1) ho += __shfl_xor(ho, off);
                if (lane == 0) P.sym_ho[k] = ho;
            }
            if (lane == 0) P.node_run_start[k] = (int64_t)base;
        }
        __syncthreads();
        if (lane < 32) {
            P.bin_nruns[k * 32 + lane] = L.bnr[lane];
            P.bin_count[k * 32 + lane] = (uint16_t)L.binc[lane];
            const unsigned nf = L.bfar[lane];
            P.bin_dist[k * 32 + lane] = nf ? (float)(sqrt((double)nf) * sp) : 0.0f;
        }
        if (lane == 0) {
            atomicAdd(&P.stats[0], examined);
            atomicAdd(&P.stats[1], (unsigned long long)nsize);
            if (COUNT) {
                atomicAdd(&P.stats[2], (unsigned long long)nsteps);
                atomicAdd(&P.stats[3], (unsigned long long)nchunks);
                P.src_work[2 * k] = nsteps;
                P.src_work[2 * k + 1] = nchunks;
            } else if (PROF) {
                atomicAdd(&P.stats[2], (unsigned long long)nsteps);
                atomicAdd(&P.stats[3], (unsigned long long)nchunks);
                for (int i = 0; i < 4; i++) atomicAdd(&P.stats[18 + i], mst[i]);
            }
            if (PROF) {
                for (int i = 0; i < 10; i++) atomicAdd(&P.stats[8 + i], cyc[i]);
                atomicAdd(&P.stats[22], cyc[10]);
                for (int i = 0; i < 3; i++) atomicAdd(&P.stats[23 + i], spst[i]);
                for (int i = 0; i < 3; i++) atomicAdd(&P.stats[26 + i], cyc[11 + i]);
                for (int i = 0; i < 3; i++) atomicAdd(&P.stats[29 + i], spst[3 + i]);
            }
            P.attrs[k * 3 + 0] = (float)nsize;
            P.attrs[k * 3 + 1] = m1f;
            P.attrs[k * 3 + 2] = m2f;
        }
        __syncthreads();
        for (int i = 0; i < 14; i++) cyc[i] = 0;
        for (int i = 0; i < 4; i++) mst[i] = 0;
        for (int i = 0; i < 6; i++) spst[i] = 0;
        MK_T(7);
    }
}

// addGridConnections (pointdata.cpp:1735-1768): bit i/4 set if the 8-neighbour in direction i is
// covered by bin i (0,4,..,28).  One thread per node.
__global__ void gridconn_kernel(int rows, const int32_t* node_cell, int64_t n, const int64_t* node_run_start,
                                const int32_t* bin_nruns, const Run* pool, uint8_t* out) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const int cell = node_cell[k];
    const int cx = cell / rows, cy = cell % rows;
    const int nx[8] = {cx + 1, cx + 1, cx, cx - 1, cx - 1, cx - 1, cx, cx + 1};
    const int ny[8] = {cy, cy + 1, cy + 1, cy + 1, cy, cy - 1, cy - 1, cy - 1};
    int64_t off = node_run_start[k];
    uint8_t gc = 0;
    for (int b = 0; b < 32; b++) {
        const int nr = bin_nruns[k * 32 + b];
        if ((b & 3) == 0) {
            const int i = b >> 2;
            for (int r = 0; r < nr; r++) {
                Run ru = pool[off + r];
                bool hit;
                if (ru.y0 == ru.y1 && ru.x0 != ru.x1) hit = (ny[i] == ru.y0 && nx[i] >= ru.x0 && nx[i] <= ru.x1);
                else if (ru.x0 == ru.x1 && ru.y0 != ru.y1) hit = (nx[i] == ru.x0 && ny[i] >= ru.y0 && ny[i] <= ru.y1);
                else if (ru.x0 == ru.x1) hit = (nx[i] == ru.x0 && ny[i] == ru.y0);
                else {
                    int dy = (ru.y1 > ru.y0) ? 1 : -1;
                    hit = nx[i] >= ru.x0 && nx[i] <= ru.x1 && (ny[i] - ru.y0) == dy * (nx[i] - ru.x0);
                }
                if (hit) { gc |= (uint8_t)(1 << i); break; }
            }
        }
        off += nr;
    }
    out[k] = gc;
}

} // namespace dmx
