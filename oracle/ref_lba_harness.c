/*
 * ref_lba_harness.c -- drives the reference's OWN local-BA functions
 * (src/local_bundle_adjustment.c: matrix_add, zero_*, invert_block_diagonal_matrix,
 * initialize_random_matrix, and gemmini_functions_cpu.h's matmul2, all compiled from their
 * sources by oracle/Makefile into oracle/_ref/libmv_ref_lba.so) through main()'s chunk loop
 * (:128-250), whose result C is a local of main and cannot be read otherwise.  Only the loop
 * structure is restated here; every arithmetic operation is the reference's.
 */
#include <stdbool.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

void matrix_add(float *A, float *B, float *C, int rows, int cols, int strideA, int strideB, int strideC, float alpha,
                float beta);
void invert_block_diagonal_matrix(float *matrix, int dim, int block_size);
void zero_block_diagonal_matrix(float *matrix, int dim, int block_size);
void zero_matrix(float *matrix, int rows, int cols);
void initialize_random_matrix(float *matrix, int rows, int cols);
void matmul2(size_t dim_I, size_t dim_J, size_t dim_K, const float *A, const float *B, const float *D, float *C,
             size_t stride_A, size_t stride_B, size_t stride_D, size_t stride_C, float A_scale_factor,
             float B_scale_factor, float D_scale_factor, bool transpose_A, bool transpose_B);

/* C [(6P+1)^2] accumulates over L / LC chunks; J from initialize_random_matrix as in main */
void ref_lba_schur_main(int P, int L, int LC, float *C) {
    const int S = 6 * P + 1, TL = 3 * LC, FW = 10, FH = 2;
    float *A = calloc((size_t)TL * TL, sizeof(float)), *B = calloc((size_t)S * TL, sizeof(float));
    float *BA = calloc((size_t)S * TL, sizeof(float)), *Jc = calloc((size_t)P * LC * FH * FW, sizeof(float));
    float H[100] = {0}; /* main's H_factor is uninitialised: +0 here (matmul2 multiplies it by 0) */
    for (int c0 = 0; c0 < L; c0 += LC) {
        zero_block_diagonal_matrix(A, TL, 3);
        zero_matrix(B, S, TL);
        initialize_random_matrix(Jc, FH * P * LC, FW);
        for (int ci = 0; ci < LC; ci++)
            for (int p = 0; p < P; p++) {
                const int pi = p * 6, li = ci * 3;
                float *J = Jc + (size_t)(p * ci) * FH * FW;
                matmul2(FW, FW, FH, J, J, H, H, FH, FH, FW, FW, 1, 1, 0, false, true);
                matrix_add(H, A + li * (TL + 1), A + li * (TL + 1), 3, 3, FW, TL, TL, 1, 1);
                matrix_add(H + 3, B + pi + li * S, B + pi + li * S, 6, 3, FW, S, S, 1, 1);
                matrix_add(H + FW - 1, B + (li + 1) * S - 1, B + (li + 1) * S - 1, 1, 3, FW, S, S, 1, 1);
                matrix_add(H + 3 * (FW + 1), C + pi * (S + 1), C + pi * (S + 1), 6, 6, FW, S, S, 1, 1);
                matrix_add(H + 4 * FW - 1, C + (pi + 1) * S - 1, C + (pi + 1) * S - 1, 1, 6, FW, S, S, 1, 1);
            }
        invert_block_diagonal_matrix(A, TL, 3);
        matmul2(TL, 6 * P, TL, A, B, BA, BA, TL, S, S, S, 1, 1, 0, false, false);
        matmul2(6 * P, 6 * P, TL, B, BA, C, C, S, S, S, S, -1, 1, 1, true, false);
    }
    free(A);
    free(B);
    free(BA);
    free(Jc);
}
