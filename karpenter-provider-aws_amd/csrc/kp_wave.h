// Wave-level reductions for gfx950 (64-lane wavefronts), shared by the Solve / consolidation evaluation and the launch
// kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Full-wave reductions without LDS permutes: DPP inside each 16-lane row (quad xor 1, quad xor 2, half-row mirror, row
// mirror leave every lane of a row holding the row's value), then the four row values combined through readlane.  The
// result is wave-uniform.  Callers run with the whole wave active.
// Debug builds (-DKPSIM_DEVICE_DEBUG) check the whole-wave precondition: with an inactive lane, update_dpp's bound
// lanes read 0 and a readlane of an inactive row would return a stale value, so a divergent call site fails loudly.
#ifdef KPSIM_DEVICE_DEBUG
#include <cassert>
#define KP_ASSERT_FULL_WAVE() assert(__builtin_amdgcn_read_exec() == ~0ull)
#else
#define KP_ASSERT_FULL_WAVE() ((void)0)
#endif

template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t x) {
    return ((uint64_t)dpp32<CTRL>((uint32_t)(x >> 32)) << 32) | dpp32<CTRL>((uint32_t)x);
}
__device__ __forceinline__ uint64_t rlane64(uint64_t x, int l) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
}
constexpr int kDppQuadXor1 = 0xB1, kDppQuadXor2 = 0x4E, kDppRowHalfMirror = 0x141, kDppRowMirror = 0x140;
template <class F>
__device__ __forceinline__ uint32_t wave_reduce32(uint32_t x, F f) {
    KP_ASSERT_FULL_WAVE();
    x = f(x, dpp32<kDppQuadXor1>(x));
    x = f(x, dpp32<kDppQuadXor2>(x));
    x = f(x, dpp32<kDppRowHalfMirror>(x));
    x = f(x, dpp32<kDppRowMirror>(x));
    uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)x, 0);
    r = f(r, (uint32_t)__builtin_amdgcn_readlane((int)x, 16));
    r = f(r, (uint32_t)__builtin_amdgcn_readlane((int)x, 32));
    return f(r, (uint32_t)__builtin_amdgcn_readlane((int)x, 48));
}
// Inclusive prefix sum over the 64 lanes (lane i gets x_0 + .. + x_i), all DPP: a Hillis-Steele scan inside each row
// (row_shr 1, 2, 4, 8; lanes shifted out of the row read 0), then row_bcast:15 adds the last lane of rows 0 / 2 to rows
// 1 / 3 and row_bcast:31 adds lane 31 to rows 2 and 3 (the GFX9 broadcast controls; gfx950 keeps them).
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp32z(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xF, true);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ uint64_t dpp64z(uint64_t x) {
    return ((uint64_t)dpp32z<CTRL, ROWS>((uint32_t)(x >> 32)) << 32) | dpp32z<CTRL, ROWS>((uint32_t)x);
}
__device__ __forceinline__ uint32_t wave_scan_add32(uint32_t x) {
    KP_ASSERT_FULL_WAVE();
    x += dpp32z<0x111, 0xF>(x);
    x += dpp32z<0x112, 0xF>(x);
    x += dpp32z<0x114, 0xF>(x);
    x += dpp32z<0x118, 0xF>(x);
    x += dpp32z<0x142, 0xA>(x);
    x += dpp32z<0x143, 0xC>(x);
    return x;
}
__device__ __forceinline__ uint64_t wave_scan_add64(uint64_t x) {
    KP_ASSERT_FULL_WAVE();
    x += dpp64z<0x111, 0xF>(x);
    x += dpp64z<0x112, 0xF>(x);
    x += dpp64z<0x114, 0xF>(x);
    x += dpp64z<0x118, 0xF>(x);
    x += dpp64z<0x142, 0xA>(x);
    x += dpp64z<0x143, 0xC>(x);
    return x;
}
template <class F>
__device__ __forceinline__ uint64_t wave_reduce64(uint64_t x, F f) {
    KP_ASSERT_FULL_WAVE();
    x = f(x, dpp64<kDppQuadXor1>(x));
    x = f(x, dpp64<kDppQuadXor2>(x));
    x = f(x, dpp64<kDppRowHalfMirror>(x));
    x = f(x, dpp64<kDppRowMirror>(x));
    uint64_t r = rlane64(x, 0);
    r = f(r, rlane64(x, 16));
    r = f(r, rlane64(x, 32));
    return f(r, rlane64(x, 48));
}
