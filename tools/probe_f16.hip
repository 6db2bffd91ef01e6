// Numerics probe (gfx950): does the f32 -> f16 conversion keep f16 subnormals, and does the f16
// MFMA take them as inputs?  The one-pass fp16 screen's window bound depends on it: with
// gradual underflow a converted component is off by at most max(2^-11 |x|, 2^-25); flushed, by
// |x| for |x| < 2^-14.  Prints, per test value x: the converted bits, and the MFMA sum of
// 16 copies of x * 1.0 (one row of a 32x32x16 product with B = 1).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void probe(const float *xs, int n, unsigned *cvt_bits, float *mfma_out) {
    const int lane = threadIdx.x;
    for (int i = 0; i < n; i++) {
        const float x = xs[i];
        unsigned r;
        asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(x));
        if (lane == 0) cvt_bits[i] = r;
        // A: lane l holds row l & 31, k = 8 (l >> 5) .. +7 -- every element x (as converted)
        const _Float16 h = __builtin_bit_cast(_Float16, (unsigned short)(r & 0xffff));
        f16x8 a, b;
        for (int k = 0; k < 8; k++) {
            a[k] = h;
            b[k] = (_Float16)1.0f;
        }
        f32x16 c = {};
        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
        if (lane == 0) mfma_out[i] = c[0];
    }
}

int main() {
    const float xs[] = {1.0f,      0.0625f,   6.103515625e-05f, 3.0517578125e-05f, 1e-5f,   1e-6f, 1e-7f,
                        5.96e-08f, 2.98e-08f, 1e-8f,             -1e-6f,            -3e-5f, 0.0f};
    const int n = sizeof xs / sizeof xs[0];
    float *dx, *dm;
    unsigned *db;
    if (hipMalloc(&dx, sizeof xs) || hipMalloc(&dm, sizeof xs) || hipMalloc(&db, n * 4)) return 2;
    if (hipMemcpy(dx, xs, sizeof xs, hipMemcpyHostToDevice)) return 2;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dx, n, db, dm);
    if (hipDeviceSynchronize()) return 3;
    unsigned bits[32];
    float m[32];
    if (hipMemcpy(bits, db, n * 4, hipMemcpyDeviceToHost) || hipMemcpy(m, dm, n * 4, hipMemcpyDeviceToHost)) return 2;
    int flushed = 0;
    for (int i = 0; i < n; i++) {
        const _Float16 h = __builtin_bit_cast(_Float16, (unsigned short)(bits[i] & 0xffff));
        const float back = (float)h;
        printf("x=% .9g  f16=0x%04x (%.9g)  mfma(16 x x)=%.9g  expect %.9g\n", xs[i], bits[i] & 0xffff, back, m[i],
               16.0f * back);
        if (xs[i] != 0.f && fabsf(xs[i]) < 6.1e-5f && fabsf(xs[i]) > 6e-8f && back == 0.f) flushed++;
        if (m[i] != 16.0f * back) flushed += 100;
    }
    printf("f16 subnormals: %s\n", flushed == 0 ? "PRESERVED by cvt and MFMA" : "FLUSHED somewhere");
    return 0;
}
