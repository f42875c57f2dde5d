/* amx_hip_experimental.h -- entry points compiled only into an AMX_EXPERIMENTAL=1 build
 * (python -m amp_extensions_amd._build with AMX_EXPERIMENTAL=1 in the environment).
 *
 * They are measured-slower (or equal) alternates of the default f16x3 forward, kept for A/B
 * experiments (round 4, the limb format 14.05 vs 15.83 M env-steps/s on one
 * box, profiles/r04c_limbs_ab.txt; round 5, the one-launch forward, profiles/r05*_ab.txt).  The default library does not export them; the export test and
 * __graft_entry__.build() check include/amx_hip.h only.  The experimental build also enables
 * amx_set_out_tile 2 / 3 (the output layer's LDS-DMA ring tile) and 4 (256 x 224 stream-K tiles),
 * and the 128 x 256 RFF tile (RFF_TILE=1). */
#pragma once
#include "amx_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Limb-format activations (csrc/experimental/amx_gemm_lb.hip; DeviceEnsemble act_format="limbs"): every
 * activation row is stored as scaled fp16 limb pairs in the fp32 row's bytes -- granules of 16
 * columns [limb0 16 x f16 | limb1 16 x f16], value = (limb0 + limb1) * 2^(E - 14) -- with one
 * exponent E per row and chunk: slot 0 = the x0 slice [0, k0), slot c >= 1 = columns
 * [k0 + 128 (c - 1), k0 + 128 c) of the hidden slices (row_exp [g][slots][rexp_ld]).  Each value
 * is split once, by its producer; the consumer's K loop copies bytes (LDS-DMA) and rescales its
 * fp32 accumulators by 2^(E_prev - E_next) at chunk boundaries.
 * amx_assemble_input_limbs: x0 (amx_assemble_input's values, dynamics.py:225-227) as limbs +
 * slot 0 of every model (stride_m 0: one copy in model 0's rows, read by every model through
 * k_shared = k0). */
int amx_assemble_input_limbs(amx_ctx* ctx, const void* ob, const void* act, int in_dtype, float* act_buf,
                             long long stride_m, int ldk, int B, int* row_exp, long long strideRexp,
                             void* stream);
/* A/B option of the limb forward's K loop: 0 (default) register-staged, 1 LDS-DMA (slower). */
int amx_set_lb_stage(amx_ctx* ctx, int stage);
/* One dense-connect hidden layer of every member (BasicMLP.forward, dynamics.py:427-430) on
 * limb-format rows: reads columns [0, K) (chunks 0 .. (K - k0)/128), writes relu(x W^T + b) as
 * limbs into columns [col_off, col_off + N) and their chunk exponents into row_exp_out (the
 * slot of the first output chunk, group 0; strideRexp / rexp_ld as row_exp).  W2 / w_exp:
 * amx_split_f16x2 images.  k_shared: 0 or k0 (x0 read from group 0's rows). */
int amx_gemm_bias_act_lb(amx_ctx* ctx, int groups, int rows, int N, int K, const float* A, int lda,
                         long long strideA, const uint16_t* W2, long long strideW2, const int* w_exp,
                         long long strideWexp, const float* bias, long long strideBias, float* C, int ldc,
                         long long strideC, int col_off, int act, const int* row_exp, long long strideRexp,
                         long long rexp_ld, int* row_exp_out, int k0, int k_shared, void* stream);
/* The output layer + un-normalisation (DynamicsModel.forward, dynamics.py:228-232) on
 * limb-format rows: preds = (x W^T + b) * sd_d + mu_d, fp32. */
int amx_gemm_out_unnorm_lb(amx_ctx* ctx, int groups, int rows, int n_valid, int K, const float* A, int lda,
                           long long strideA, const uint16_t* W2, long long strideW2, const int* w_exp,
                           long long strideWexp, const float* bias, long long strideBias, float* preds, int ldp,
                           long long strideP, const int* row_exp, long long strideRexp, long long rexp_ld, int k0,
                           int k_shared, void* stream);

/* The one-launch f16x3 forward (csrc/experimental/amx_fwd.hip; DeviceEnsemble forward_mode
 * "fused", bench --forward fused): measured equal to the per-layer launches at the N = 8 share
 * (307-310 vs 307 us per forward, profiles/r05m_ab.txt) and slower at 8192 lanes, where it does
 * not apply -- every layer boundary is an HBM-bound burst of the slice's stores in both forms.
 * The whole f16x3 ensemble forward in one launch (BasicMLP.forward over the dense-concat rows,
 * milo/milo/dynamics.py:422-433, + the un-normalisation :231-232): the n_hidden
 * amx_gemm_bias_act_h3 launches and amx_gemm_out_unnorm_h3 of one forward, bit-identical to them
 * (same K order, limb products and row exponents), with one workgroup per block of rows of one
 * member for every layer (csrc/amx_fwd.hip: no grid-wide step between layers).
 * A [groups][rows][lda] fp32: columns [0, k0) = x0 (slot 0 of row_exp filled, k_shared = 0 or
 * k0 as amx_gemm_bias_act_h3), hidden slice i written at column k0 + i*hidden; W2 / w_exp /
 * bias: arrays of n_hidden + 1 device pointers (layer i: the amx_fwd_weight_image of its
 * amx_split_f16x2 image, N = hidden rows, K_i = k0 + i*hidden; the output layer: N = n_out_pad,
 * K_out = k0 + n_hidden*hidden; w_exp / bias [groups][N] as for the per-layer launches);
 * preds [groups][rows][ldp] (group stride strideP) un-normalised with the context's
 * normalizers; row_exp slots 1..n_hidden are written as the per-layer chain leaves them.
 * hidden = 512, n_hidden <= 8, k0 % 64 == 0, n_out_pad in {128, 256} with S in
 * (n_out_pad - 128, n_out_pad].  amx_forward_h3_rows: the rows per workgroup it uses for
 * groups x rows -- one workgroup per CU of 64, 80 or 96 rows (4096 / 5120 / 6144 lanes x 4
 * members on 256 CUs) -- and 0 for other shapes (then amx_forward_h3 returns AMX_E_INVAL:
 * use the per-layer launches). */
int amx_forward_h3_rows(amx_ctx* ctx, int groups, int rows);
/* The fragment order amx_forward_h3 reads its weights in: W2 [groups][N][K/16][2][16] (the
 * amx_split_f16x2 image) -> W2f [groups][N/16][K/32][limb 2][lane 64][8 f16], lane = 32 * k-granule
 * + 16 * half + row within the 16-row block (one 1 KB contiguous load per MFMA fragment).
 * Same size as W2; N % 16 == 0, K % 32 == 0. */
int amx_fwd_weight_image(amx_ctx* ctx, int groups, int N, int K, const uint16_t* W2, uint16_t* W2f, void* stream);
int amx_forward_h3(amx_ctx* ctx, int groups, int rows, int k0, int hidden, int n_hidden, float* A, int lda,
                   long long strideA, const uint16_t* const* W2, const int* const* w_exp,
                   const float* const* bias, int n_out_pad, float* preds, int ldp, long long strideP,
                   int* row_exp, long long strideRexp, int k_shared, void* stream);

#ifdef __cplusplus
}
#endif
