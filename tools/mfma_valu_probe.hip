// Issue probe (timing only): how v_mfma_i32_32x32x32_i8 and independent VALU work share one SIMD.
// Each wave runs ITER iterations of { 2 MFMAs on two independent accumulator chains, NV VALU
// ops on unrelated registers (v_max3_i32 chains), optionally NL ds_read_b128 }; s_memtime brackets
// the loop.  Launched with WPS waves per SIMD (256-thread workgroups, one per CU per wave slot).
// Prints cycles per MFMA pair per wave and the implied MFMA-pipe busy fraction of the SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

template <int NV, int NL>
__global__ __launch_bounds__(256) void probe(int iters, unsigned long long *out, int *sink) {
    __shared__ i32x4 lds[1024];
    const int t = threadIdx.x;
    lds[t] = i32x4{t, t + 1, t + 2, t + 3};
    __syncthreads();
    i32x4 a = {t, 1, 2, 3}, b = {3, t, 1, 2};
    i32x16 c0 = {}, c1 = {};
    int v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = t + k;
    i32x4 l = {};
    i32x4 r[3][2];  // B fragments: NL = 2 reads them from LDS 3 steps ahead (as the match kernels)
#pragma unroll
    for (int j = 0; j < 3; j++) {
        r[j][0] = NL ? lds[(t + 64 * j) & 1023] : b;
        r[j][1] = NL ? lds[(t + 64 * j + 32) & 1023] : b;
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it += 3) {
#pragma unroll
        for (int j = 0; j < 3; j++) {
            c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, r[j][0], c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, r[j][1], c1, 0, 0, 0);
            if constexpr (NL > 0) {
                r[j][0] = lds[(t + 64 * (it + j)) & 1023];
                r[j][1] = lds[(t + 64 * (it + j) + 32) & 1023];
            }
#pragma unroll
            for (int k = 0; k < NV; k++) {
                int q;
                asm volatile("v_max3_i32 %0, %1, %2, %3" : "=v"(q) : "v"(v[k & 7]), "v"(v[(k + 1) & 7]), "v"(v[(k + 3) & 7]));
                v[k & 7] = q;
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    int s = c0[0] + c1[3] + l[0];
#pragma unroll
    for (int k = 0; k < 8; k++) s += v[k];
    if (s == 0x12345678) sink[0] = s;
    if ((t & 63) == 0) out[blockIdx.x * 4 + (t >> 6)] = t1 - t0;
}

template <int NV, int NL>
void run(int wps, int cus) {
    const int blocks = cus * wps, iters = 3999;
    unsigned long long *d;
    int *sink;
    hipMalloc(&d, blocks * 4 * 8);
    hipMalloc(&sink, 4);
    hipLaunchKernelGGL((probe<NV, NL>), dim3(blocks), dim3(256), 0, 0, iters, d, sink);
    hipLaunchKernelGGL((probe<NV, NL>), dim3(blocks), dim3(256), 0, 0, iters, d, sink);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(blocks * 4);
    hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    double sum = 0;
    for (auto x : h) sum += (double)x;
    const double cyc = sum / h.size() / iters;  // per iteration (2 MFMAs) per wave
    // SIMD MFMA busy: wps waves x 2 MFMAs x 32 cycles per `cyc` cycles of each wave
    printf("NV=%2d NL=%d waves/SIMD=%d: %.1f cycles per MFMA pair per wave -> MFMA pipe %.0f %%\n", NV, NL, wps, cyc,
           100.0 * wps * 64.0 / cyc);
    hipFree(d);
    hipFree(sink);
}

int main() {
    int dev = 0, cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    for (int wps = 1; wps <= 2; wps++) {
        run<0, 0>(wps, cus);
        run<10, 0>(wps, cus);
        run<14, 0>(wps, cus);
        run<0, 2>(wps, cus);
        run<6, 2>(wps, cus);
        run<10, 2>(wps, cus);
        run<14, 2>(wps, cus);
    }
    return 0;
}
