// common.hpp -- shared device-side definitions for the dmx HIP kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "../host/geometry.hpp"

namespace dmx {

constexpr int WAVE = 64;

// Error flags raised by kernels (bitwise OR into a device word; the host maps them to status codes).
enum KernelError : int {
    KERR_GAP_CAPACITY = 1,     // sieve gap list exceeded LDS capacity
    KERR_BLOCK_CAPACITY = 2,   // per-depth block list exceeded LDS capacity
    KERR_STAGE_CAPACITY = 4,   // per-source run staging exceeded scratch capacity
    KERR_POOL_CAPACITY = 8,    // global run pool exhausted
    KERR_BIN_MISMATCH = 16,    // whichbin produced a bin outside the octant (should never happen)
    KERR_LEVELS = 32,          // BFS depth exceeded the level histogram
    KERR_FRONTIER = 64,        // BFS frontier buffer overflow
};

// Per-cell word uploaded to HBM: bit 0 FILLED, bits 1..7 cropped-segment count (<=127),
// bits 8..31 offset of the cell's first segment.
__host__ __device__ inline uint32_t pack_cell(bool filled, uint32_t nseg, uint32_t off) {
    return (off << 8) | (nseg << 1) | (filled ? 1u : 0u);
}
__device__ __forceinline__ bool cell_filled(uint32_t w) { return w & 1u; }
__device__ __forceinline__ int cell_nseg(uint32_t w) { return (int)((w >> 1) & 127u); }
__device__ __forceinline__ int cell_seg_off(uint32_t w) { return (int)(w >> 8); }

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

} // namespace dmx
