/*
 * ref_harness.c -- exports thin wrappers around the reference's header-only
 * code so tests can call it through ctypes.  Compiled by oracle/Makefile ONLY
 * where /root/reference exists; output goes to oracle/_ref/ (git-ignored).
 * The reference sources are used where they lie (include paths), never copied.
 */
#include <stdbool.h>
#include "gemmini_functions_cpu.h" /* include/gemmini_functions_cpu.h:14-124 */

/* C[I][J] += A[I][K] . B[J][K]^T  -- the all-pairs match shape */
void ref_matmul_nt(int I, int J, int K, const float *A, const float *B, float *C) {
    matmul((size_t)I, (size_t)J, (size_t)K, A, B, C, (size_t)K, (size_t)K, (size_t)J, 1.0f, 1.0f, false, true);
}
