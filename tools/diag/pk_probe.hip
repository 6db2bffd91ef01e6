// pk_probe.hip -- diagnosis only (tools/diag): do gfx950's packed-FP32 VOP3P instructions
// give the same bits as the scalar VALU for the operand-select / negate forms the SLP vectoriser
// emitted in k_pose_intended's 8-point QR -- alone, and while other kernels run on another stream?
// Each thread runs chains of 4 dependent packed ops on its own inputs and checks every result
// against v_fma_f32 / v_mul_f32 / moves on the same halves.  Counts of mismatching words go to one
// vector atomic per thread.  Built by tools/diag/build.sh with -fno-slp-vectorize (the reference
// side must stay scalar).
#include <hip/hip_runtime.h>

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float ufl(unsigned u) {  // a float in [-2, 2), 23 random mantissa bits
    return __uint_as_float(0x40000000u | (u >> 9)) - 3.0f;
}

template <int F>
__device__ __forceinline__ f2 pk(f2 a, f2 b, f2 c) {
    f2 d;
    if constexpr (F == 0) asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    if constexpr (F == 1) asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    if constexpr (F == 2) asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    if constexpr (F == 3)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1] neg_lo:[1,0,0] neg_hi:[1,0,0]"
                     : "=v"(d) : "v"(a), "v"(b), "v"(c));
    if constexpr (F == 4)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] neg_lo:[1,0,0] neg_hi:[1,0,0]"
                     : "=v"(d) : "v"(a), "v"(b), "v"(c));
    if constexpr (F == 5) asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    if constexpr (F == 6) asm volatile("v_pk_mov_b32 %0, %1, %2 op_sel:[1,0]" : "=v"(d) : "v"(a), "v"(b));
    if constexpr (F == 7) asm volatile("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(d) : "v"(a), "v"(b));
    if constexpr (F == 8) asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    if constexpr (F == 9) asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,1]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    if constexpr (F == 10) asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1]" : "=v"(d) : "v"(a), "v"(b));
    if constexpr (F == 11) asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[0,1]" : "=v"(d) : "v"(a), "v"(b));
    if constexpr (F == 12)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,0,1]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    if constexpr (F == 13)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %3 neg_lo:[1,0,0] neg_hi:[1,0,0]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    if constexpr (F == 14) asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    if constexpr (F == 15) asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0]" : "=v"(d) : "v"(a), "v"(b));
    return d;
}

template <int F>
__device__ __forceinline__ f2 ref(f2 a, f2 b, f2 c) {
    f2 d;
    if constexpr (F == 0) d = f2{__builtin_fmaf(a.x, b.x, c.x), __builtin_fmaf(a.y, b.y, c.y)};
    if constexpr (F == 1) d = f2{__builtin_fmaf(a.x, b.x, c.x), __builtin_fmaf(a.x, b.y, c.y)};
    if constexpr (F == 2) d = f2{__builtin_fmaf(a.y, b.x, c.x), __builtin_fmaf(a.y, b.y, c.y)};
    if constexpr (F == 3) d = f2{__builtin_fmaf(-a.x, b.x, c.x), __builtin_fmaf(-a.y, b.x, c.y)};
    if constexpr (F == 4) d = f2{__builtin_fmaf(-a.x, b.y, c.x), __builtin_fmaf(-a.y, b.y, c.y)};
    if constexpr (F == 5) d = f2{a.x * b.x, a.y * b.y};
    if constexpr (F == 6) d = f2{a.y, b.x};
    if constexpr (F == 7) d = f2{a.x - b.x, a.y - b.y};
    if constexpr (F == 8) d = f2{__builtin_fmaf(a.x, b.y, c.x), __builtin_fmaf(a.y, b.y, c.y)};
    if constexpr (F == 9) d = f2{__builtin_fmaf(a.x, b.x, c.y), __builtin_fmaf(a.y, b.y, c.y)};
    if constexpr (F == 10) d = f2{a.x * b.y, a.y * b.y};
    if constexpr (F == 11) d = f2{a.x + b.y, a.y + b.y};
    if constexpr (F == 12) d = f2{__builtin_fmaf(a.x, b.y, c.x), __builtin_fmaf(a.y, b.x, c.y)};
    if constexpr (F == 13) d = f2{__builtin_fmaf(-a.x, b.x, c.x), __builtin_fmaf(-a.y, b.y, c.y)};
    if constexpr (F == 14) d = f2{__builtin_fmaf(a.x, b.x, c.x), __builtin_fmaf(a.y, b.x, c.y)};
    if constexpr (F == 15) d = f2{a.y * b.x, a.y * b.y};
    return d;
}

// samples[0] counts recorded mismatches; record k (< 32) at samples + 1 + 8 k: form, lane half, a, b,
// c (the halves used), got, expected -- as raw bits
template <int F>
__global__ __launch_bounds__(256) void k_pk_probe(int iters, unsigned seed, unsigned *bad, unsigned *samples) {
    unsigned s = seed ^ (blockIdx.x * 256u + threadIdx.x) * 0x9E3779B9u;
    unsigned nbad = 0;
    for (int it = 0; it < iters; it++) {
        s = s * 1664525u + 1013904223u;
        const unsigned s1 = s * 747796405u + 2891336453u, s2 = s1 * 747796405u + 2891336453u;
        f2 a = {ufl(s), ufl(s1)}, b = {ufl(s2), ufl(s ^ s2)}, c = {ufl(s1 ^ s2), ufl(s + s1)};
        f2 y = a;
#pragma unroll
        for (int k = 0; k < 4; k++) {  // a dependent chain, as the QR's column updates are
            const f2 in = y;
            const f2 x = pk<F>(in, b, c);
            y = ref<F>(in, b, c);
            const bool bx = __float_as_uint(x.x) != __float_as_uint(y.x), by = __float_as_uint(x.y) != __float_as_uint(y.y);
            nbad += bx + by;
            if (bx | by) {
                const unsigned q = atomicAdd(samples, 1u);
                if (q < 32) {
                    unsigned *o = samples + 1 + 10 * q;
                    o[0] = F | (bx ? 0x100u : 0u) | (by ? 0x200u : 0u);
                    o[1] = __float_as_uint(in.x);
                    o[2] = __float_as_uint(in.y);
                    o[3] = __float_as_uint(b.x);
                    o[4] = __float_as_uint(b.y);
                    o[5] = __float_as_uint(c.x);
                    o[6] = __float_as_uint(c.y);
                    o[7] = __float_as_uint(x.x);
                    o[8] = __float_as_uint(x.y);
                    o[9] = (blockIdx.x << 8) | threadIdx.x;
                }
            }
            y = y * 0.25f;  // keep the chain finite: restart from the reference's value
        }
    }
    if (nbad) atomicAdd(bad + F, nbad);
}

extern "C" int mv_dbg_pk_probe(int form, int blocks, int iters, unsigned seed, unsigned *bad, unsigned *samples,
                               hipStream_t s) {
    switch (form) {
#define L(F) case F: hipLaunchKernelGGL(k_pk_probe<F>, dim3(blocks), dim3(256), 0, s, iters, seed, bad, samples); break;
        L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8) L(9) L(10) L(11) L(12) L(13) L(14) L(15)
#undef L
        default: return -1;
    }
    return (int)hipGetLastError();
}
