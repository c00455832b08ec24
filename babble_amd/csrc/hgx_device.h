// Device helpers shared by the libhgx HIP translation units (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace hgx {

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

__device__ __forceinline__ uint64_t group_mask(int gs, int grp) {
    return (gs >= 64) ? ~0ull : (((1ull << gs) - 1ull) << (gs * grp));
}

// order LDS accesses of one wave (lanes exchange data through LDS without a block barrier)
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

}  // namespace hgx
