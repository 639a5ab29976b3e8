// Row-streaming bandwidth probe for eval_rows' access pattern (tools only, not the product):
// one workgroup per row of a Q x G fp32 matrix, NT threads, U float4 loads per thread in
// flight, a per-row sum written out.  Built and timed by tools/rowread_bw.py.
#include <hip/hip_runtime.h>
#include <cstdint>

template <int NT, int U>
__global__ __launch_bounds__(NT) void rowread_kernel(const float* __restrict__ d, int64_t G, float* __restrict__ out) {
    const float4* r4 = (const float4*)(d + blockIdx.x * G);
    const int nv = (int)(G >> 2);
    float s = 0.f;
    for (int g0 = 0; g0 < nv; g0 += NT * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int g = g0 + u * NT + threadIdx.x;
            v[u] = r4[g < nv ? g : nv - 1];
        }
#pragma unroll
        for (int u = 0; u < U; u++) s += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    if (s == 1234.5f) out[blockIdx.x] = s;  // keeps the loads; never true on the probe's data
}

extern "C" int rowread(const float* d, int64_t Q, int64_t G, float* out, int variant, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    switch (variant) {
        case 0: hipLaunchKernelGGL((rowread_kernel<256, 4>), dim3(Q), dim3(256), 0, s, d, G, out); break;
        case 1: hipLaunchKernelGGL((rowread_kernel<256, 8>), dim3(Q), dim3(256), 0, s, d, G, out); break;
        case 2: hipLaunchKernelGGL((rowread_kernel<256, 16>), dim3(Q), dim3(256), 0, s, d, G, out); break;
        case 3: hipLaunchKernelGGL((rowread_kernel<512, 4>), dim3(Q), dim3(512), 0, s, d, G, out); break;
        case 4: hipLaunchKernelGGL((rowread_kernel<1024, 4>), dim3(Q), dim3(1024), 0, s, d, G, out); break;
        default: return 1;
    }
    return hipGetLastError() == hipSuccess ? 0 : 2;
}
