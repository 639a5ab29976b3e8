// common.h — shared helpers for the libreidmi HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include "reidmi.h"

#define REIDMI_API extern "C" __attribute__((visibility("default")))

namespace reidmi {

enum Status : int { OK = 0, EINVAL_ = 1, EHIP = 2, ECAP = 3 };

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define RM_CHECK_HIP(expr)                                                                  \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return ::reidmi::fail(::reidmi::EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define RM_REQUIRE(cond, msg)                                               \
    do {                                                                    \
        if (!(cond)) return ::reidmi::fail(::reidmi::EINVAL_, std::string(msg)); \
    } while (0)

// After a launch: report launch-configuration errors immediately.
#define RM_LAUNCHED() RM_CHECK_HIP(hipGetLastError())

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// bf16 <-> f32 by bit manipulation (RNE; inputs here are finite).
__device__ __forceinline__ unsigned short f2bf_bits(float f) {
    unsigned int u = __float_as_uint(f);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (unsigned short)(u >> 16);
}
__device__ __forceinline__ float bf2f_bits(unsigned short h) { return __uint_as_float(((unsigned int)h) << 16); }

// fp16 (IEEE binary16) round-trip with RNE, matching numpy's npy_float_to_half.
__device__ __forceinline__ unsigned short f2h_bits(float f) {
    _Float16 h = (_Float16)f;
    return __builtin_bit_cast(unsigned short, h);
}
__device__ __forceinline__ float h2f_bits(unsigned short b) { return (float)__builtin_bit_cast(_Float16, b); }

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

}  // namespace reidmi
