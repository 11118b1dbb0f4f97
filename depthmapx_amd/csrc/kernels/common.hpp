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

} // namespace dmx
