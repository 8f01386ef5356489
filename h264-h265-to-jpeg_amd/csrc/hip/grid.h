// Workgroup -> (tile, picture) order for the 2-D grids (x: tile of a picture, y: picture) of the
// kernels whose neighbouring tiles share lines: K0 (consecutive TB records write neighbouring
// residual rows), K3 SAO (CTB halos), K4c, K5b, K5d (tiles of one picture's symbol stream).
// Measured on hevc1080 per 1024 pictures (tools/gpu_ab.sh, same box): K0 -6 %, SAO -4 %, K4c
// -5 %, K5b/K5d -4-5 %.  Pure streaming kernels keep the plain order: K4a (+37 %) and K4e
// (+14 %) got slower with it -- the dispatcher's round-robin spreads one picture's rows over
// all XCDs and HBM channels at once, which is what a read-once stream wants; HEVC deblocking
// was neutral.
#pragma once
#ifdef __HIP__
#include <hip/hip_runtime.h>
#define H2J_GRID_FN __host__ __device__ __forceinline__
#else
#define H2J_GRID_FN inline  // plain C++ (tests/test_grid_remap.py checks the mapping on the host)
#endif

// XCD-aware order (guide §5.5 T1).  The dispatcher deals consecutive workgroups of a launch
// round-robin to the 8 XCDs, each with a private L2, so tiles that share halo rows / columns
// or 128-B lines (a CTB and its neighbours, consecutive 8x8-block tiles) would each be fetched
// once per XCD.  The linear workgroup id is remapped so that the workgroups one XCD receives
// (orig % 8 labels them) cover one contiguous range of (picture, tile) ids.  Bijective for any
// grid size n (q = n / 8, r = n % 8); it changes only where a tile runs, never a result -- no
// kernel using it depends on dispatch order.  -DH2J_NO_XCD_REMAP restores the plain order
// (A/B builds).
H2J_GRID_FN unsigned xcd_remap(unsigned orig, unsigned n) {
    const unsigned xcd = orig & 7u, q = n >> 3, r = n & 7u;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

#ifdef __HIP__
struct GridPos {
    int x, y;
};
__device__ __forceinline__ GridPos xcd_grid_pos() {
#ifdef H2J_NO_XCD_REMAP
    return GridPos{static_cast<int>(blockIdx.x), static_cast<int>(blockIdx.y)};
#else
    const unsigned gx = gridDim.x;
    const unsigned id = xcd_remap(blockIdx.y * gx + blockIdx.x, gx * gridDim.y);
    return GridPos{static_cast<int>(id % gx), static_cast<int>(id / gx)};
#endif
}
#endif
