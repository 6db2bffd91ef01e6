// Diagnosis: sustained int8 MFMA throughput of v_mfma_i32_32x32x32_i8 against v_mfma_i32_16x16x64_i8
// on random operands, every CU busy (2 waves per SIMD, independent accumulator chains, operands in
// registers), the operands perturbed every iteration so nothing is constant.  Results land in a
// sink buffer (vector stores).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

extern "C" __global__ __launch_bounds__(512, 1) void mfma32_probe(const int *__restrict__ seed, int iters, int *__restrict__ sink) {
    const int t = threadIdx.x + blockIdx.x * blockDim.x;
    i32x4 a = {seed[(t * 7) & 4095], seed[(t * 13) & 4095], seed[(t * 17) & 4095], seed[(t * 19) & 4095]};
    i32x4 b = {seed[(t * 23) & 4095], seed[(t * 29) & 4095], seed[(t * 31) & 4095], seed[(t * 37) & 4095]};
    i32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
            c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, a, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, b, c3, 0, 0, 0);
        }
        a = a ^ (i32x4){it, it * 3, it * 5, it * 7};
        b = b ^ (i32x4){it * 11, it * 13, it * 17, it * 19};
    }
    int s = 0;
#pragma unroll
    for (int q = 0; q < 16; q++) s += c0[q] ^ c1[q] ^ c2[q] ^ c3[q];
    sink[t] = s;
}

// 16x16x64: 64 MFMAs of 32768 ops per iteration (twice the 32x32 kernel's ops: the driver counts each)
extern "C" __global__ __launch_bounds__(512, 1) void mfma16_probe(const int *__restrict__ seed, int iters, int *__restrict__ sink) {
    const int t = threadIdx.x + blockIdx.x * blockDim.x;
    i32x4 a = {seed[(t * 7) & 4095], seed[(t * 13) & 4095], seed[(t * 17) & 4095], seed[(t * 19) & 4095]};
    i32x4 b = {seed[(t * 23) & 4095], seed[(t * 29) & 4095], seed[(t * 31) & 4095], seed[(t * 37) & 4095]};
    i32x4 c[16] = {};
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
#pragma unroll
            for (int k = 0; k < 16; k += 4) {
                c[k] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c[k], 0, 0, 0);
                c[k + 1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, a, c[k + 1], 0, 0, 0);
                c[k + 2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, a, c[k + 2], 0, 0, 0);
                c[k + 3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, b, c[k + 3], 0, 0, 0);
            }
        }
        a = a ^ (i32x4){it, it * 3, it * 5, it * 7};
        b = b ^ (i32x4){it * 11, it * 13, it * 17, it * 19};
    }
    int s = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) s += c[k][0] ^ c[k][1] ^ c[k][2] ^ c[k][3];
    sink[t] = s;
}

extern "C" int mv_dbg_mfma_probe(int shape, int blocks, int iters, const int *seed, int *sink, void *stream) {
    if (shape == 32)
        hipLaunchKernelGGL(mfma32_probe, dim3(blocks), dim3(512), 0, (hipStream_t)stream, seed, iters, sink);
    else
        hipLaunchKernelGGL(mfma16_probe, dim3(blocks), dim3(512), 0, (hipStream_t)stream, seed, iters, sink);
    return (int)hipGetLastError();
}
