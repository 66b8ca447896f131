// pk_dpp_probe.hip -- minimal kernel for tests/test_pk_hazard.py: the attention-dot
// pattern of csrc/gat_infer.hip (gat_layer_infer_kernel step 2) in isolation.  Each
// 16-lane row accumulates two dot products s1, s2 of an LDS row with two weight
// vectors (two independent float32 chains: with packed-FP32 instructions allowed the
// compiler pairs them into v_pk_mul_f32 / v_pk_add_f32), then sums them over its 16
// lanes with four DPP steps and stores them.  Built twice from this one source
// (Makefile `hazard`): PROBE_NAME=trx_probe_packed with packed FP32 allowed, and
// PROBE_NAME=trx_probe_scalar with -packed-fp32-ops, as the shipped library is built.
#include <hip/hip_runtime.h>

#define PDPP(v, ctrl) __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xf, 0xf, false))

__device__ __forceinline__ float row_sum16(float v) {
    v = v + PDPP(v, 0xB1);   // quad_perm [1,0,3,2]
    v = v + PDPP(v, 0x4E);   // quad_perm [2,3,0,1]
    v = v + PDPP(v, 0x141);  // row_half_mirror
    v = v + PDPP(v, 0x140);  // row_mirror
    return v;
}

// one workgroup of 256 threads per block of rows; x [rows][256], w1/w2 [256];
// out [rows][2].  Row r of the block is read by 16-lane row (r % 4) of wave (r / 4) % 4.
#define PCAT2(a, b) a##b
#define PCAT(a, b) PCAT2(a, b)
#define PROBE_KERNEL PCAT(PROBE_NAME, _kernel)
__global__ void __launch_bounds__(256) PROBE_KERNEL(const float* __restrict__ x, const float* __restrict__ w1,
                                                    const float* __restrict__ w2, float* __restrict__ out,
                                                    int rows_per_block) {
    __shared__ __attribute__((aligned(16))) float xs[64 * 256];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int sub = lane >> 4, sl = lane & 15;
    const int r0 = blockIdx.x * rows_per_block;
    for (int v = tid; v < rows_per_block * 64; v += 256)
        reinterpret_cast<float4*>(xs)[v] = reinterpret_cast<const float4*>(x + (size_t)r0 * 256)[v];
    __syncthreads();
    float4 sa[4], da[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        sa[m] = *reinterpret_cast<const float4*>(w1 + 4 * sl + 64 * m);
        da[m] = *reinterpret_cast<const float4*>(w2 + 4 * sl + 64 * m);
    }
    for (int i0 = 4 * wave; i0 < rows_per_block; i0 += 16) {
        const int i = i0 + sub;
        float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const float4 x4 = *reinterpret_cast<const float4*>(xs + i * 256 + 4 * sl + 64 * m);
            s1 += (x4.x * sa[m].x + x4.y * sa[m].y) + (x4.z * sa[m].z + x4.w * sa[m].w);
            s2 += (x4.x * da[m].x + x4.y * da[m].y) + (x4.z * da[m].z + x4.w * da[m].w);
        }
        s1 = row_sum16(s1);
        s2 = row_sum16(s2);
        if (sl == 0) {
            out[(size_t)(r0 + i) * 2] = s1;
            out[(size_t)(r0 + i) * 2 + 1] = s2;
        }
    }
}

extern "C" int PROBE_NAME(const float* x, const float* w1, const float* w2, float* out, int rows, void* stream) {
    const int rpb = 64;
    if (rows % rpb) return -1;
    hipLaunchKernelGGL(PROBE_KERNEL, dim3(rows / rpb), dim3(256), 0, static_cast<hipStream_t>(stream), x, w1, w2,
                       out, rpb);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
