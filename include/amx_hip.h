/*
 * amx_hip.h — C ABI of the MI355X-native learned-dynamics rollout engine.
 *
 * This is the drop-in boundary for ONE hot path of dhruvsreenivas/amp_extensions:
 * the gym_simenv learned-dynamics step (4-model dense-MLP ensemble), the MILO
 * random-Fourier-feature MMD cost + ensemble-disagreement bonus, the AMP/GAIL
 * least-squares discriminator reward and the humanoid3d fall/horizon termination.
 * Each entry point names the reference interface it replaces (paths relative to
 * the reference repository root).
 *
 * Conventions
 *   - Every buffer argument is a DEVICE pointer owned by the caller, except where a
 *     comment says "host".  Nothing is retained after a call returns, except the
 *     small configuration copied by amx_set_* into context-owned device memory.
 *   - Every launching call takes a hipStream_t (passed as void* so this header
 *     needs no HIP include) and is asynchronous on it.  No call allocates, frees
 *     or synchronises on the launch path, so a caller may capture them in a graph.
 *   - Return value: AMX_OK (0) or a negative AMX_E_* code.  No exception crosses
 *     the ABI.  amx_last_error() returns a thread-local message for the last
 *     failing call on the calling thread.
 *   - Thread safety: one amx_ctx per device; calls on one context are not
 *     re-entrant; distinct contexts/devices are independent.
 *   - Row padding: GEMM operands/outputs have a row count that is a multiple of
 *     AMX_ROW_TILE (128); K of every GEMM is a multiple of AMX_K_TILE (32); leading
 *     dimensions are multiples of 4 floats; pointers are 16-byte aligned.
 *     amx_layout() reports the padded widths the engine expects.
 */
#ifndef AMX_HIP_H
#define AMX_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AMX_ABI_VERSION 2
#define AMX_ROW_TILE 128
#define AMX_K_TILE 32
#define AMX_MAX_MODELS 8
#define AMX_MAX_BODIES 32
#define AMX_MT_STATE_BYTES 2512  /* one numpy-legacy MT19937 state (amx_mt_seed) */

enum {
  AMX_OK = 0,
  AMX_E_INVAL = -1,   /* bad argument (shape, alignment, null pointer) */
  AMX_E_HIP = -2,     /* HIP runtime error (launch, memcpy) */
  AMX_E_NOMEM = -3,   /* device allocation failed */
  AMX_E_STATE = -4    /* context not configured for this call */
};

enum { AMX_SHAPE_SPHERE = 0, AMX_SHAPE_CAPSULE = 1, AMX_SHAPE_BOX = 2 };
enum { AMX_ACT_NONE = 0, AMX_ACT_RELU = 1 };
enum { AMX_IN_F64 = 0, AMX_IN_F32 = 1 };
enum { AMX_DISC_LEAST_SQUARES = 0, AMX_DISC_LOG_LIKELIHOOD = 1 };

typedef struct amx_ctx amx_ctx;

/* ---- context ------------------------------------------------------------------ */

/* Replaces the sizes SimEnv/DynamicsEnsemble read at construction:
 * gym-simenv/gym_simenv/envs/sim_env.py:66-67 (state/action size),
 * milo/milo/dynamics.py:19-79 (num_models, hidden_sizes) and
 * milo/milo/linear_cost.py:23-62 (feature_dim).  n_hidden hidden layers of width
 * `hidden`, dense-connected (BasicMLP, milo/milo/dynamics.py:394-433). */
amx_ctx* amx_create(int device, int S, int A, int n_models, int hidden, int n_hidden, int feat_dim);
int amx_destroy(amx_ctx* ctx);
const char* amx_last_error(void);
int amx_abi_version(void);

/* Padded layout the engine expects (host outputs):
 *   k0_pad   = round_up(S + A, 32)   width of the [s~, a~] block of the activation row
 *   ldk      = k0_pad + n_hidden*hidden  activation row length (dense-concat buffer)
 *   n_out_pad= round_up(S, 128)      output rows of the padded last-layer weight
 *   k_rff_pad= round_up(2*S, 32)     width of the float32 [s, s'] cost input row   */
int amx_layout(const amx_ctx* ctx, int* k0_pad, int* ldk, int* n_out_pad, int* k_rff_pad);

/* Normalizers (host pointers, copied).  Contract of AmpDataset.get_transformations,
 * milo/milo/datasets.py:23-43: means and mean-absolute-deviation+1e-8 scales, in
 * the order DynamicsModel.forward consumes them (milo/milo/dynamics.py:225-232). */
int amx_set_normalizers(amx_ctx* ctx, const float* mu_s, const float* sd_s, const float* mu_a,
                        const float* sd_a, const float* mu_d, const float* sd_d);

/* Fall-termination configuration (host pointers, copied).  Replaces SimEnv.__init__'s
 * fall-body tables and ctrl flags, gym-simenv/gym_simenv/envs/sim_env.py:83-115, and
 * is_done/check_velocity's parameters, :164-173, :259-268.  body_id[i] is the
 * character body index; p0/p1 are BodyDefs Param0/Param1 (radius = 0.5*p0, capsule
 * height = p1).  pos_dim/rot_dim: per-body pose feature widths (3 and 6). */
int amx_set_termination(amx_ctx* ctx, int n_bodies, const int32_t* body_id, const int32_t* shape,
                        const double* p0, const double* p1, int record_all_world,
                        int record_world_root_pos, int pos_dim, int rot_dim, int horizon,
                        int vel_check, int vel_offset, double vel_thresh, int record_vel_as_pos,
                        double sampling_rate);

/* ---- ensemble forward --------------------------------------------------------- */

/* State assembly for DynamicsModel.forward, milo/milo/dynamics.py:216-230:
 * x0 = [(float(s)-mu_s)/sd_s, (float(a)-mu_a)/sd_a, 0-pad] written at column 0 of
 * every model's activation row (act_buf[m][b][0:k0_pad], m < n_models).
 * in_dtype = AMX_IN_F64 (SimEnv's float64 ob, sim_env.py:155-156) or AMX_IN_F32. */
int amx_assemble_input(amx_ctx* ctx, const void* ob, const void* act, int in_dtype, float* act_buf,
                       long long stride_m, int ldk, int B, void* stream);
/* The same assembly for the f16x3 GEMM path: also writes slot 0 of the row exponents
 * (row_exp[m][slot][b], slot stride slot_stride >= B, model stride strideRexp; the layout of
 * amx_row_exponents) from max |x0| and resets slots 1..n_slots-1, for rows b < B.
 * stride_m = 0: x0 is written once (model 0's rows) and the f16x3 GEMMs read it for every
 * model (their k_shared); the exponent slots are still written for every model.
 * Member-blocked layout (slot_stride = Bq < B, stride_m = 0, B = M' x Bq with M' <= M): lane b
 * belongs to member block g = b / Bq (the sampler's one-member-per-lane forward), its x0 is row b
 * and its exponents go to row b % Bq of block g's slots only (g * strideRexp + slot * Bq). */
int amx_assemble_input_rexp(amx_ctx* ctx, const void* ob, const void* act, int in_dtype, float* act_buf,
                            long long stride_m, int ldk, int B, int* row_exp, long long strideRexp,
                            long long slot_stride, int n_slots, void* stream);

/* Grouped fp32 GEMM on MFMA with fused bias (+ReLU) epilogue: for g < groups,
 * C_g[r][col_off + n] = act(sum_k A_g[r][k] * W_g[n][k] + bias_g[n]).
 * One dense-connect hidden layer of all ensemble members at once
 * (BasicMLP.forward, milo/milo/dynamics.py:427-430: relu(fc(x)); x = cat[x, h]);
 * also the Discriminator hidden layers, milo/milo/gail_cost.py:18-42.
 * rows % 128 == 0, N % 128 == 0, K % 32 == 0. */
int amx_gemm_bias_act(amx_ctx* ctx, int groups, int rows, int N, int K, const float* A, int lda,
                      long long strideA, const float* W, int ldw, long long strideW,
                      const float* bias, long long strideBias, float* C, int ldc, long long strideC,
                      int col_off, int act, void* stream);

/* Last dense layer + output un-normalisation (BasicMLP.forward :432 then
 * DynamicsModel.forward :231-232): preds_g[r][n] = (sum_k A W + b[n]) * sd_d[n] + mu_d[n]
 * for n < n_valid (=S); W_g is padded to round_up(n_valid,128) rows. */
int amx_gemm_out_unnorm(amx_ctx* ctx, int groups, int rows, int n_valid, int K, const float* A,
                        int lda, long long strideA, const float* W, int ldw, long long strideW,
                        const float* bias, long long strideBias, float* preds, int ldp,
                        long long strideP, void* stream);

/* ---- bf16x6: the same fp32 GEMMs on the bf16 matrix pipe ------------------------
 * Each fp32 operand is split exactly into three bf16 limbs (x = x0 + x1 + x2) and a*b is
 * summed as the six limb products of degree <= 2 in fp32 MFMA accumulators: fp32-level
 * error (the dropped terms are <= 2^-23 |ab|), 2.67x fewer matrix-pipe cycles than the f32
 * MFMA.  Same semantics, layouts and epilogues as amx_gemm_bias_act / amx_gemm_out_unnorm
 * (BasicMLP.forward, milo/milo/dynamics.py:422-433 + DynamicsModel.forward :231-232); only
 * the weight operand differs: W3 is the image written by amx_split_bf16x3.  K % 16 == 0.
 *
 * amx_split_bf16x3: W [groups][rows][K] fp32 (row stride ldw, group stride strideW) ->
 * W3 [groups][rows][K/16][3][16] bf16 bits (row stride 3K, group stride strideW3). */
int amx_split_bf16x3(amx_ctx* ctx, int groups, int rows, int K, const float* W, int ldw,
                     long long strideW, uint16_t* W3, long long strideW3, void* stream);
int amx_gemm_bias_act_x6(amx_ctx* ctx, int groups, int rows, int N, int K, const float* A, int lda,
                         long long strideA, const uint16_t* W3, long long strideW3, const float* bias,
                         long long strideBias, float* C, int ldc, long long strideC, int col_off,
                         int act, void* stream);
int amx_gemm_out_unnorm_x6(amx_ctx* ctx, int groups, int rows, int n_valid, int K, const float* A,
                           int lda, long long strideA, const uint16_t* W3, long long strideW3,
                           const float* bias, long long strideBias, float* preds, int ldp,
                           long long strideP, void* stream);

/* bf16x6 form of amx_rff_features (RBFLinearCost.get_rep, milo/milo/linear_cost.py:64-71):
 * W3 = amx_split_bf16x3 image of the [F][K] RFF weight; same epilogue and outputs. */
int amx_rff_features_x6(amx_ctx* ctx, int rows, int n_valid, int F, int K, const float* x, int ldx,
                        const uint16_t* W3, const float* b, float scale, float* phi, int ldphi,
                        double* col_partials, const uint8_t* row_mask, void* stream);

/* ---- f16x3: the same fp32 GEMMs as two scaled fp16 limbs, three products ---------------
 * Each fp32 operand is scaled by a power of two (per weight row / per activation row) and
 * split into two fp16 limbs (11 + 11 significant bits); a*b = a0b0 + a0b1 + a1b0 in fp32
 * MFMA accumulators.  The per-term error (<= ~2^-22 |ab|) adds up like sqrt(K) while the
 * fp32 accumulation's grows like K, so the GEMM error equals an fp32 GEMM's for K >= ~64
 * (tools/x6_accuracy.py); 3 MFMA per 32x32x16 block instead of bf16x6's 6.  Same
 * semantics, layouts and epilogues as amx_gemm_bias_act / amx_gemm_out_unnorm
 * (BasicMLP.forward, milo/milo/dynamics.py:422-433 + DynamicsModel.forward :231-232).
 *
 * amx_split_f16x2: W [groups][rows][K] fp32 -> W2 [groups][rows][K/16][2][16] fp16 bits
 * (row stride 2K) scaled by 2^(14 - E_r), E_r = w_exp[g][r] (max_k |W| < 2^E_r).
 * Row exponents of A: row_exp [groups][slots][rows] int32 (group stride strideRexp, slot
 * stride = rows); a GEMM scales row r by 2^(14 - max over slots 0..rexp_slots-1).
 * amx_row_exponents writes slot 0 from A's first K columns and resets slots 1..n_slots-1;
 * amx_gemm_bias_act_h3 with row_exp_out (the slot of the columns it writes; nullable)
 * max-es the exponents of its output rows into it, so a dense-concat chain of layers
 * (layer i reads slots 0..i, writes slot i+1) needs no other pass.  K % 16 == 0.
 * k_shared (multiple of 32, 0 = off): A's first k_shared columns are read from group 0's rows
 * for every group -- the ensemble's x0 slice assembled once (amx_assemble_input_rexp with
 * stride_m = 0) instead of one copy per model; each group's row_exp slot 0 still holds its
 * exponents. */
int amx_split_f16x2(amx_ctx* ctx, int groups, int rows, int K, const float* W, int ldw,
                    long long strideW, uint16_t* W2, long long strideW2, int* w_exp,
                    long long strideWexp, void* stream);
int amx_row_exponents(amx_ctx* ctx, int groups, int rows, int K, const float* A, int lda,
                      long long strideA, int* row_exp, long long strideRexp, int n_slots,
                      void* stream);
int amx_gemm_bias_act_h3(amx_ctx* ctx, int groups, int rows, int N, int K, const float* A, int lda,
                         long long strideA, const uint16_t* W2, long long strideW2, const int* w_exp,
                         long long strideWexp, const float* bias, long long strideBias, float* C,
                         int ldc, long long strideC, int col_off, int act, const int* row_exp,
                         long long strideRexp, int rexp_slots, int* row_exp_out, int k_shared,
                         void* stream);
int amx_gemm_out_unnorm_h3(amx_ctx* ctx, int groups, int rows, int n_valid, int K, const float* A,
                           int lda, long long strideA, const uint16_t* W2, long long strideW2,
                           const int* w_exp, long long strideWexp, const float* bias,
                           long long strideBias, float* preds, int ldp, long long strideP,
                           const int* row_exp, long long strideRexp, int rexp_slots, int k_shared,
                           void* stream);

/* f16x3 form of amx_rff_features (RBFLinearCost.get_rep, milo/milo/linear_cost.py:64-71):
 * W2/w_exp = amx_split_f16x2 image of the [F][K] RFF weight, row_exp [rows] = exponents of x's
 * rows (amx_step_rexp, or amx_row_exponents with one slot); same epilogue and outputs. */
int amx_rff_features_h3(amx_ctx* ctx, int rows, int n_valid, int F, int K, const float* x, int ldx,
                        const uint16_t* W2, const int* w_exp, const int* row_exp, const float* b, float scale,
                        float* phi, int ldphi, double* col_partials, const uint8_t* row_mask, void* stream);

/* SimEnv's reset noise (reset_args noise_bef_rot, noise_min, noise_max, radian, rot_vel_w_pose,
 * vel_noise, interp, knee_rot; run.py:113-117) = DeepMimicCore's cKinCharacter::AddNoise
 * (anim/KinCharacter.cpp:340-470) applied to the kinematic pose / velocity at the reset time.
 * The draws come from Philox (the C++ core's std::default_random_engine stream cannot be
 * reproduced) or, for tests, from an injected [B][ld_draws] table of uniforms in [0, 1):
 * RandomRotatePoseVel's draws at [0, AMX_NOISE_ROT_SLOTS), AddNoisePoseVel's (pose elements,
 * then velocity elements) after them. */
#define AMX_NOISE_ROT_SLOTS 48
typedef struct amx_reset_noise {
  int noise_bef_rot;
  double noise_min, noise_max, radian;
  int rot_vel_w_pose, vel_noise;
  double interp;
  int knee_rot;
} amx_reset_noise;
int amx_motion_states_noise(amx_ctx* ctx, const double* times, int B, int flags, const amx_reset_noise* noise,
                            const double* draws, long long ld_draws, uint64_t seed, double* ob, long long ldo,
                            void* stream);
int amx_reset_lanes_motion_noise(amx_ctx* ctx, const uint8_t* mask, const double* times, uint64_t seed,
                                 double time_max, int flags, const amx_reset_noise* noise, const double* draws,
                                 long long ld_draws, const double* ob_src, double* ob_out, int32_t* num_steps,
                                 int32_t* model_idx, int32_t* reset_count, double* t_out, int B, void* stream);
/* ---- reference-motion resets (SimEnv.reset -> DeepMimicCore reset_time, §8f #2) ----------
 * amx_set_motion: host blob (copied; amp_extensions_amd/motion.py build_blob): header[16]
 *   {J, D, F, loop, duration, -, -, -, cycle_delta xyz, ground_pad, ...}, joints [J][8]
 *   {type (0 revolute, 3 fixed, 4 spherical, 5 root), parent, param offset, param size,
 *   attach xyz, -}, bodies [J][8] {shape (0 box, 1 capsule, 2 sphere), attach xyz, Param0-2,
 *   valid}, frame times [F], post-processed frames [F][D], frame velocities [F][D]
 *   (cMotion::Load, deepmimic/deepmimic/DeepMimicCore/anim/Motion.cpp:104-188, 415-442).
 *   Requires S == 1 + 15 J (CtController pose + velocity layout, sim/CtController.cpp:305-319).
 * amx_motion_states: ob[b] = the state recorded after reset_time(times[b]) (motion pose and
 *   velocity at t, plane placement, ground resolve, CtController::BuildStatePose/Vel);
 *   flags: 1 RecordWorldRootPos, 2 RecordWorldRootRot, 4 RecordAllWorld, 8 no ground resolve
 *   (reset_args['resolve'] = False: SceneSimChar::ResetSceneTime skips ResolveCharGroundIntersect,
 *   deepmimic/deepmimic/DeepMimicCore/scenes/SceneSimChar.cpp:714-716).
 * amx_reset_lanes_motion: amx_reset_lanes with those states; t = times[b] or
 *   uniform(0, time_max) from Philox(seed, lane, reset#) (sim_env.py:276); time_max <= 0 means the
 *   clip length (sim_env.py:77; reset_args['time_max'] with custom_time); t_out nullable. */
int amx_set_motion(amx_ctx* ctx, const double* blob, long long n);
double amx_motion_duration(const amx_ctx* ctx);
int amx_motion_states(amx_ctx* ctx, const double* times, int B, int flags, double* ob, long long ldo,
                      void* stream);
int amx_reset_lanes_motion(amx_ctx* ctx, const uint8_t* mask, const double* times, uint64_t seed,
                           double time_max, int flags, const double* ob_src, double* ob_out, int32_t* num_steps,
                           int32_t* model_idx, int32_t* reset_count, double* t_out, int B, void* stream);

/* AMP observation features (SceneImitateAMP::BuildAMPObs, deepmimic/deepmimic/DeepMimicCore/
 * scenes/SceneImitateAMP.cpp:352-475; the discriminator input of the original AMP agent):
 * [pose(cur), pose(prev), vel(cur), vel(prev)] in the current heading frame, amx_amp_obs_size
 * doubles per row (humanoid3d: 226).  Needs amx_set_motion's character tables.
 *   amx_state_amp_obs:  from recorded SimEnv states (s_prev, s_cur) [B][lds] — the agent's
 *                       features of a transition (RecordAMPObsAgent, :154-165);
 *   amx_motion_amp_obs: from the clip at times[b] - dt and times[b] (RecordAMPObsExpert,
 *                       :167-193; dt = 1 / UpdateRate).
 * local_root = enable_amp_obs_local_root (default false, :29). */
int amx_amp_obs_size(const amx_ctx* ctx);
int amx_state_amp_obs(amx_ctx* ctx, const double* s_prev, const double* s_cur, long long lds, int B,
                      int local_root, double* out, long long ldo, void* stream);
int amx_motion_amp_obs(amx_ctx* ctx, const double* times, double dt, int B, int local_root, double* out,
                       long long ldo, void* stream);
/* amx_state_amp_obs written as float32 cost-input rows (the AMP-feature discriminator's
 * input), zero-padded from amx_amp_obs_size up to ldo. */
int amx_state_amp_rows(amx_ctx* ctx, const double* s_prev, const double* s_cur, long long lds, int B,
                       int local_root, float* out, long long ldo, void* stream);

/* ---- NPG policy update (the rollout's learner; mjrl/mjrl/algos/npg_cg.py:113-199) ----
 * Policy: mjrl MLP(S -> 32 -> 32 -> A, tanh) + log_std (mjrl/mjrl/policies/gaussian_mlp.py),
 * parameters packed in the reference's flat order (W1, b1, W2, b2, W3, b3, log_std; fp32,
 * amx_npg_param_count(S, A) floats).  obs [N][ldo] / act [N][lda] are fp64 or fp32
 * (AMX_IN_*); the policy reads float32(obs) as the reference does (gaussian_mlp.py:112-117).
 * amx_npg_pass writes one fp64 partial per block of rows_per_block rows (multiple of 32):
 *   mode 0 (VPG):  grad of mean(exp(LL_new - LL_old) * adv) at new == old
 *                  (BatchREINFORCE.flat_vpg, batch_reinforce.py:58-62)            -> [blocks][P]
 *   mode 1 (FVP):  J^T diag(2/(2 sigma^2 + 1e-8)) J vec / N, the mean-network block of
 *                  NPG.HVP (npg_cg.py:87-106; log_std block and damping: caller)  -> [blocks][P]
 *   mode 2 (EVAL): sum of exp(LL_vec - LL_theta) * adv and of the per-sample mean_kl
 *                  terms (surr_after / kl_old_new, npg_cg.py:181-183)             -> [blocks][2]
 * amx_npg_reduce sums the partials over blocks in block order (deterministic). */
long long amx_npg_param_count(int S, int A);
int amx_npg_pass(amx_ctx* ctx, int mode, int N, const void* obs, int obs_dtype, long long ldo,
                 const void* act, int act_dtype, long long lda, const double* adv, const float* theta,
                 const float* vec, int rows_per_block, double* partials, void* stream);
int amx_npg_reduce(amx_ctx* ctx, const double* partials, int blocks, int P, double* out, void* stream);
/* The same with a gate: gate = the CG state of amx_npg_cg_init / _step ({rdotr, live}); with
 * live == 0 the pass and the reduction return at once (every block reads the flag), so the FVP
 * products of a solve that stopped early cost two empty launches, not a pass over the batch
 * (cg_solve.py:19-20 breaks the loop there). */
int amx_npg_pass_gated(amx_ctx* ctx, int mode, int N, const void* obs, int obs_dtype, long long ldo,
                       const void* act, int act_dtype, long long lda, const double* adv, const float* theta,
                       const float* vec, int rows_per_block, double* partials, const double* gate, void* stream);
int amx_npg_reduce_gated(amx_ctx* ctx, const double* partials, int blocks, int P, double* out, const double* gate,
                         void* stream);
/* amx_npg_pass_gated with the policy's forward at theta cached per sample: hcache [N][64] fp32
 * (H1 = tanh(W1 x + b1) | H2 = tanh(W2 H1 + b2)), 16-byte aligned.  Mode 0 (VPG) writes it; mode 1
 * (FVP, fp32 observations) reads it instead of recomputing layers 1-2 at theta -- valid only for
 * the theta and observations of the VPG pass that wrote it (npg_cg.py:123-135: the CG's ten
 * Fisher-vector products share them).  The FVP partials are bit-identical to the uncached pass. */
int amx_npg_pass_ex(amx_ctx* ctx, int mode, int N, const void* obs, int obs_dtype, long long ldo, const void* act,
                    int act_dtype, long long lda, const double* adv, const float* theta, const float* vec,
                    int rows_per_block, double* partials, const double* gate, float* hcache, void* stream);

/* The conjugate-gradient solve of NPG (mjrl/mjrl/utils/cg_solve.py:3-23) on the device, one
 * workgroup per call, fixed-order fp64 reductions, no host round trip between iterations.
 * amx_npg_cg_init: x = 0, r = p = b, p32 = float32(p), state = {r.r, 1 (live)}.
 * amx_npg_cg_step, after h = amx_npg_reduce(amx_npg_pass(FVP, vec = p32)):
 *   z = h + [log_std block: curv * p32] + damping * p   (NPG.HVP's return, npg_cg.py:105)
 *   v = rdotr / p.z; x += v p; r -= v z; rr = r.r; p = r + (rr / rdotr) p; rdotr = rr;
 *   live = rdotr >= residual_tol (cg_solve's break: a finished solve leaves x/r/p unchanged);
 *   p32 = float32(p) for the next product.  curv [A]: d^2 mean_kl / d log_std^2.  P <= 16384. */
/* d^2 mean_kl / d log_std^2 per action at new == old (NPG.HVP's log_std block,
 * gaussian_mlp.py:144-155): curv[d] = (8 s^2 - 4 s 1e-8) / (2 s + 1e-8)^2, s = exp(log_std[d])^2,
 * log_std = theta[P - A ..]. */
int amx_npg_curvature(amx_ctx* ctx, const float* theta, int P, int A, double* curv, void* stream);
/* The NPG step after the CG (npg_cg.py:141-163) in one workgroup: gdot = vpg . npg; use_alpha
 * (const_learn_rate): n_step_size = alpha^2 gdot, else alpha = sqrt(|n_step_size / (gdot + 1e-20)|);
 * new_theta = float32(theta + alpha npg) with the log_std block clamped at min_log_std
 * (gaussian_mlp.py:71-94); scal = {alpha, n_step_size, gdot}.  P <= 16384. */
int amx_npg_apply_step(amx_ctx* ctx, int P, int A, const double* vpg, const double* npg, const float* theta,
                       int use_alpha, double alpha, double n_step_size, float min_log_std, float* new_theta,
                       double* scal, void* stream);
/* amx_npg_reduce (the FVP pass's partials, the same summation order) and amx_npg_cg_step
 * (cg_solve.py:3-23: one iteration after the Fisher-vector product) in two launches over the
 * chip: the column sums with z and the blocks' p.z parts; then x, r, p and the state, every block
 * forming v = rdotr / p.z and r'.r' itself in one fixed order (so p.z and r.r sum in another order
 * than amx_npg_cg_step's).  The residual and the state alternate between two caller buffers
 * (iteration i reads r_in / state_in and writes r_out / state_out; the next swaps them: every
 * block reads all of r); x, p, p32 are updated in place.  A stopped solve (state_in[1] == 0)
 * copies r and the state over and changes nothing else.  work: caller-owned fp64
 * [amx_npg_cg_tail_work(P)], no state kept between calls.  Replaces round 4's
 * amx_npg_reduce_cg_step (one launch, the step by the last-arriving block). */
long long amx_npg_cg_tail_work(int P);
int amx_npg_cg_tail(amx_ctx* ctx, const double* partials, int blocks, int P, int A, const double* curv,
                    double damping, double tol, double* x, const double* r_in, double* r_out, double* p, float* p32,
                    const double* state_in, double* state_out, double* work, void* stream);
/* amx_npg_cg_tail's two launches, separately: amx_npg_cg_reduce (column sums, z and the p.z
 * parts into work; skipped when state[1] == 0) and amx_npg_cg_xrp (the vector step from work:
 * x, r_in -> r_out, p, p32 in place, state_in -> state_out). */
int amx_npg_cg_reduce(amx_ctx* ctx, const double* partials, int blocks, int P, int A, const double* curv,
                      double damping, const double* p, const float* p32, const double* state, double* work,
                      void* stream);
int amx_npg_cg_xrp(amx_ctx* ctx, int P, double tol, double* x, const double* r_in, double* r_out, double* p,
                   float* p32, const double* state_in, double* state_out, const double* work, void* stream);
/* The Fisher-vector pass (mode 1, amx_npg_pass_ex with hcache) with the PREVIOUS CG iteration's
 * vector step folded into its setup: every block forms amx_npg_cg_xrp's v, r' = r_in - v z,
 * r'.r' (xrp's summation orders: the same bits) and p' = r' + (r'.r' / r.r) p_in from work (the
 * previous amx_npg_cg_reduce) and multiplies by float32(p') instead of a vec argument; the blocks
 * write x += v p_in, r_out, p_out, p32_out (their slices) and state_out {r'.r', live}.  A solve
 * stopped before (state_in[1] == 0) or by this step (r'.r' < tol) writes no partials (the gate)
 * and carries r, p and the state over.  r, p and the state alternate buffers (every block reads
 * all of them).  One CG iteration = amx_npg_pass_cg (or, first, amx_npg_pass_gated on p32) +
 * amx_npg_cg_reduce; the solve ends with one amx_npg_cg_xrp: the step's own launch is gone from
 * every iteration but the last.  Actions are not read. */
int amx_npg_pass_cg(amx_ctx* ctx, int N, const void* obs, int obs_dtype, long long ldo, const float* theta,
                    int rows_per_block, double* partials, float* hcache, double tol, double* x, const double* r_in,
                    double* r_out, const double* p_in, double* p_out, float* p32_out, const double* state_in,
                    double* state_out, const double* work, void* stream);
int amx_npg_cg_init(amx_ctx* ctx, int P, const double* b, double* x, double* r, double* p, float* p32,
                    double* state, void* stream);
/* amx_npg_cg_init + amx_npg_curvature (theta's log_std block -> curv [A]) in one launch. */
int amx_npg_cg_init_ls(amx_ctx* ctx, int P, int A, const float* theta, double* curv, const double* b, double* x,
                       double* r, double* p, float* p32, double* state, void* stream);
int amx_npg_cg_step(amx_ctx* ctx, int P, int A, const double* h, const double* curv, double damping,
                    double residual_tol, double* x, double* r, double* p, float* p32, double* state,
                    void* stream);

/* ---- step + termination ------------------------------------------------------- */

/* One batched SimEnv.step after the forward (gym-simenv/gym_simenv/envs/sim_env.py:140-173):
 * num_steps[b] += 1; ob_next[b] = ob[b] + (double)preds[model_idx[b]][b] (fp64 state,
 * fp32 model, :158); done[b] = horizon | check_collision | check_velocity (:164-268),
 * bit-exact fp64 comparisons.  Fused extras (nullable):
 *   disc[b]   = max over model pairs of ||preds_i - preds_j||_2 (compute_discrepancy,
 *               milo/milo/dynamics.py:134-143) — reuses the step's own forward;
 *   cost_in   = float32 [ob, ob_next] rows, ld = ldc (the 'ss' cost input,
 *               mjrl/mjrl/algos/batch_reinforce.py:107-113);
 *   nonfinite[b] = 1 if ob_next holds a NaN/Inf (diagnostic only; done unchanged). */
int amx_step(amx_ctx* ctx, const float* preds, int ldp, long long strideP, const int32_t* model_idx,
             const double* ob, double* ob_next, int32_t* num_steps, uint8_t* done, float* disc,
             float* cost_in, int ldc, uint8_t* nonfinite, int B, void* stream);
/* amx_step that also writes cost_rexp[b] = the exponent of the [s, s'] cost row's max |x|
 * (max < 2^e, clamped to [-100, 100]): the row_exp operand of amx_rff_features_h3. */
int amx_step_rexp(amx_ctx* ctx, const float* preds, int ldp, long long strideP, const int32_t* model_idx,
                  const double* ob, double* ob_next, int32_t* num_steps, uint8_t* done, float* disc,
                  float* cost_in, int ldc, int* cost_rexp, uint8_t* nonfinite, int B, void* stream);

/* amx_step (cost_rexp nullable: amx_step_rexp) fused with amx_reset_lanes(mask = done,
 * ob_src = ob_next) in one pass: done lanes get reset_count/model_idx/num_steps/row_out
 * and ob_out[b] = table[row] exactly as amx_reset_lanes; the others ob_out[b] = ob_next[b]
 * (from registers, no re-read).  ob_out must differ from ob_next; it may be ob (in place:
 * every lane reads its row before writing it); model_idx is read (the member of this step)
 * and, for reset lanes, rewritten.  ob_rec (nullable, a fourth buffer) receives a copy of ob
 * (a rollout's slot 0 when the carried lane states are read where the last rollout left
 * them, instead of a separate carry copy).  steps0_out (nullable):
 * receives num_steps before this step (the trajectory position of a rollout's first slot).
 * counter (nullable): *counter += counter_delta once per launch (amx_counter_add folded into a
 * captured rollout's last step; no kernel of this launch reads the counter). */
int amx_step_reset(amx_ctx* ctx, const float* preds, int ldp, long long strideP, int32_t* model_idx,
                   const double* ob, double* ob_next, int32_t* num_steps, uint8_t* done, float* disc,
                   float* cost_in, int ldc, int* cost_rexp, uint8_t* nonfinite, const double* table,
                   int R, const int32_t* rows, uint64_t seed, double* ob_out, int32_t* reset_count,
                   int32_t* row_out, int32_t* steps0_out, uint64_t* counter, long long counter_delta,
                   double* ob_rec, int B, void* stream);

/* amx_step_reset of step t (no counter advance) fused with the policy of step t + 1 on the
 * observations it produces (obs[t+1] = ob_out): one launch runs the step of 16 lanes, keeps the
 * float32 of their obs[t+1] rows on chip and runs amx_policy_act on them (Philox noise with
 * policy_seed and counter / counter_dev as amx_policy_act[_dev]; no injected noise), writing
 * act [B][A], mean and the fused x0 / row-exponent assembly exactly as amx_policy_act.  The
 * results are bit-identical to amx_step_reset followed by amx_policy_act on ob_out (the same
 * workgroup decomposition of the policy).  Replaces, per rollout step t + 1 > 0, the reference's
 * get_action call after env.step (mjrl/mjrl/samplers/core.py via milo/milo/sampler.py:48-65).
 * S <= 256 and a policy image of at most 16384 floats. */
int amx_step_reset_act(amx_ctx* ctx, const float* preds, int ldp, long long strideP, int32_t* model_idx,
                       const double* ob, double* ob_next, int32_t* num_steps, uint8_t* done, float* disc,
                       float* cost_in, int ldc, int* cost_rexp, uint8_t* nonfinite, const double* table,
                       int R, const int32_t* rows, uint64_t seed, double* ob_out, int32_t* reset_count,
                       int32_t* row_out, int32_t* steps0_out, double* ob_rec, const float* blob, int H1,
                       int H2, const double* noise_scale, uint64_t policy_seed, uint64_t counter,
                       const uint64_t* counter_dev, int eval_mode, double* act, float* mean,
                       float* x0_buf, long long stride_m, int ldk, int* row_exp, long long stride_rexp,
                       long long slot_stride, int n_slots, int B, void* stream);
/* amx_step_reset_act's occupancy, for A/B measurement: 0 (default) one 1024-thread workgroup
 * per CU at the kernel's natural register count, 1 two per CU (registers capped at 64). */
int amx_set_step_act_occupancy(amx_ctx* ctx, int two_per_cu);

/* Disagreement only (DynamicsEnsemble.get_action_discrepancy / compute_threshold,
 * milo/milo/dynamics.py:145-165). */
int amx_disagreement(amx_ctx* ctx, const float* preds, int ldp, long long strideP, float* disc,
                     int B, void* stream);

/* SimEnv.reset for masked lanes (gym-simenv/gym_simenv/envs/sim_env.py:270-285), with
 * the DeepMimicCore pose replaced by a row of a device reset-state table (documented
 * deviation).  For every lane b with mask[b] != 0 (mask NULL = all lanes):
 *   reset_count[b] += 1; model_idx[b] = reset_count[b] % n_models; num_steps[b] = 0;
 *   row = rows ? rows[b] : philox(seed, b, reset_count[b]) mod R; ob_out[b] = table[row].
 * Lanes with mask 0 copy ob_src[b] into ob_out[b] (carry; ob_src may equal ob_out).
 * row_out (nullable) receives the chosen row (-1 for carried lanes). */
int amx_reset_lanes(amx_ctx* ctx, const uint8_t* mask, const double* table, int R,
                    const int32_t* rows, uint64_t seed, const double* ob_src, double* ob_out,
                    int32_t* num_steps, int32_t* model_idx, int32_t* reset_count, int32_t* row_out,
                    int B, void* stream);

/* ---- device policy ------------------------------------------------------------ */

/* mjrl Gaussian MLP policy action (mjrl/mjrl/policies/gaussian_mlp.py:95-104 over
 * FCNetwork tanh, mjrl/mjrl/utils/fc_network.py:42-55), two hidden layers:
 *   mean = W3 tanh(W2 tanh(W1 float(ob) + b1) + b2) + b3   (float32)
 *   act  = (double)mean + noise_scale * n,  n ~ N(0,1) fp64 (philox(seed, b, counter)
 *          Box-Muller) or injected noise[b][A] (nullable).  eval_mode: act = mean.
 * The weights come as the packed image of amx_policy_pack (re-pack after each policy
 * update, e.g. after the learner's step; not per action).
 * noise_scale = exp(log_std) in fp64 (device, [A]).
 * x0_buf (nullable) fuses the ensemble's state assembly (amx_assemble_input with
 * AMX_IN_F64) for the same lanes: x0 = [(float(ob)-mu_s)/sd_s, (float(act)-mu_a)/sd_a, 0]
 * written to every model's activation row (stride_m, ldk as in amx_assemble_input; stride_m
 * 0: once, model 0's rows, the f16x3 GEMMs' shared x0 slice); row_exp (nullable, needs x0_buf)
 * additionally writes the f16x3 row-exponent slots exactly as amx_assemble_input_rexp (including
 * its member-blocked layout, slot_stride < B). */
int amx_policy_act(amx_ctx* ctx, const double* ob, int B, const float* blob, int H1, int H2,
                   const double* noise_scale, const double* noise, uint64_t seed, uint64_t counter,
                   int eval_mode, double* act, float* mean, float* x0_buf, long long stride_m, int ldk,
                   int* row_exp, long long stride_rexp, long long slot_stride, int n_slots,
                   void* stream);

/* amx_policy_act with the Philox counter = counter[0] (device memory) + counter_offset, so a
 * captured HIP graph of a rollout (step t passes offset t) draws fresh noise on every replay;
 * amx_counter_add(counter, delta) advances it on the stream (one thread, once per rollout). */
int amx_policy_act_dev(amx_ctx* ctx, const double* ob, int B, const float* blob, int H1, int H2,
                       const double* noise_scale, const double* noise, uint64_t seed,
                       const uint64_t* counter, uint64_t counter_offset, int eval_mode, double* act,
                       float* mean, float* x0_buf, long long stride_m, int ldk, int* row_exp,
                       long long stride_rexp, long long slot_stride, int n_slots, void* stream);
int amx_counter_add(amx_ctx* ctx, uint64_t* counter, long long delta, void* stream);

/* GEMM timing that works inside captured HIP graphs (ROCm has no timing-event nodes) and adds
 * no launches: with buf set (4 uint64 of device memory, zeroed by the caller), every f16x3
 * ensemble forward on this context records the device's 100 MHz realtime counter when its
 * first hidden layer starts (amx_gemm_bias_act_h3 with rexp_slots = 1: block 0, buf[0]) and,
 * when the last workgroup of its output layer (amx_gemm_out_unnorm_h3) finishes, adds the
 * elapsed ticks to buf[2] and 1 to buf[3] (buf[1]: arrival counter, left zero).  The pointer
 * is read when a launch is issued (graph capture bakes it in).  null: off. */
int amx_set_gemm_timer(amx_ctx* ctx, uint64_t* buf);

/* Split workspace of the f16x3 output layer (amx_gemm_out_unnorm_h3): at lane counts whose
 * 128 x 224 output tiles are fewer than the CUs but at least half as many (4096-7168 lanes x 4
 * members), the layer runs stream-K: one workgroup per CU, the tiles' K-tiles dealt out evenly,
 * each tile's 1-3 K segments stored raw and summed in K order by the last arriver
 * (deterministic); the hidden layers' 128 x 256 tiles split the same way below 2048 lanes.
 * amx_split_workspace_floats: floats of scratch (up to 6 partial tiles per tile, the largest
 * of the shapes above) and *n_counters uint32 counters a forward of `rows` padded lanes needs, 0 when that shape
 * does not use it.  amx_set_split_workspace registers caller-owned device memory with the
 * context (counters zeroed by the caller once; each launch leaves them zero); without it the
 * layer runs on row-block tiles.  One launch at a time per context. */
long long amx_split_workspace_floats(const amx_ctx* ctx, int groups, int rows, int* n_counters);

int amx_set_split_workspace(amx_ctx* ctx, float* scratch, long long floats, uint32_t* counters,
                            int n_counters);

/* Floats to allocate for the packed policy weight image for hidden widths H1, H2 (host query;
 * -1 on a bad argument): the image rounded up to whole 1-KiB pieces, which
 * amx_step_reset_act copies into LDS by LDS-DMA (amx_policy_pack writes the image, the tail is
 * never read as weights). */
long long amx_policy_blob_floats(const amx_ctx* ctx, int H1, int H2);

/* Pack the policy's three nn.Linear layers (W [out][in] row-major f32, b [out]; the
 * FCNetwork fc_layers, mjrl/mjrl/utils/fc_network.py:24-31) into blob (device, 16-byte
 * aligned, amx_policy_blob_floats floats): zero-padded rows in the layout amx_policy_act
 * copies into LDS with one vector pass. */
int amx_policy_pack(amx_ctx* ctx, const float* W1, const float* b1, int H1, const float* W2,
                    const float* b2, int H2, const float* W3, const float* b3, float* blob,
                    void* stream);

/* ---- MILO RFF MMD cost -------------------------------------------------------- */

/* Rows per fp64 column partial of the RFF features (round 5: 32, was 128): col_partials has
 * rows / AMX_RFF_PART_ROWS rows, so the feature pass may use 160- and 80-row tiles that fill the
 * CUs in whole rounds (40 960 rows: 512 tiles of 160 x 256; 5 120 rows: 256 tiles of 160 x 64). */
#define AMX_RFF_PART_ROWS 32

/* RBFLinearCost.get_rep (milo/milo/linear_cost.py:64-71) on MFMA:
 * phi[r][f] = cos(sum_k x[r][k] W[f][k] + b[f]) * scale, scale = (float)sqrt(2/F),
 * plus fp64 column sums of each 32-row group's valid rows (r < n_valid and (row_mask==NULL or
 * row_mask[r])) into col_partials[r/AMX_RFF_PART_ROWS][f] — the per-rank share of the global
 * feature mean of fit_cost (:84-94); amx_feature_message / amx_sum_partials add the
 * rows / AMX_RFF_PART_ROWS partial rows in order.  rows % 128 == 0, F % 128 == 0. */
int amx_rff_features(amx_ctx* ctx, int rows, int n_valid, int F, int K, const float* x, int ldx,
                     const float* W, int ldw, const float* b, float scale, float* phi, int ldphi,
                     double* col_partials, const uint8_t* row_mask, void* stream);

/* Deterministic ordered sum of n_parts rows of fp64 partials -> out[F] (fp64). */
int amx_sum_partials(amx_ctx* ctx, const double* partials, int n_parts, int F, double* out,
                     void* stream);

/* fit_cost closed form (milo/milo/linear_cost.py:84-94) after the cross-rank sum:
 * phi_pi = (float)(phi_sum / count); w = phi_pi - phi_e; mmd[0] = dot(w, w) (fp32).
 * count = 0: the count is read from phi_sum[F] (the all-reduced [sum phi | count] message). */
int amx_mmd_fit(amx_ctx* ctx, const double* phi_sum, double count, const float* phi_e, int F,
                float* w, float* mmd, void* stream);

/* Per-sample MILO reward with pessimism (RBFLinearCost.get_costs + get_bonus_costs,
 * milo/milo/linear_cost.py:96-103, 111-152; reward = -cost, batch_reinforce.py:144):
 *   v = clamp(phi[n].w, c_min, c_max); dh = min(disc[n]/thr, 1); bonus = dh*c_min;
 *   ipm = (1-lambda)*v; wb = lambda*bonus; reward = -(ipm - wb).
 * ipm/wbonus outputs are nullable (info['ipm'], info['bonus']). */
int amx_mmd_reward(amx_ctx* ctx, const float* phi, int ldphi, const float* w, int F, const float* disc,
                   float thr, double lambda_b, float c_min, float c_max, float* reward, float* ipm,
                   float* wbonus, int n, void* stream);

/* Same with cost_range=None (linear_cost.py:103, 138-139): v = phi[n].w unclamped,
 * bonus = disc[n] (raw disagreement); ipm/wb/reward as above. */
int amx_mmd_reward_raw(amx_ctx* ctx, const float* phi, int ldphi, const float* w, int F, const float* disc,
                       double lambda_b, float* reward, float* ipm, float* wbonus, int n, void* stream);

/* get_expert_cost (milo/milo/linear_cost.py:105-109): partial fp64 sums over row
 * blocks of clamp(phi_E[r].w, c_min, c_max); out[0] = sum (fp64; out holds 1 + 1024
 * doubles).  mean_out (nullable) receives the finished cost in fp32:
 * (float)(1 - lambda_b) * (float)(sum / n).  Uses the resident expert features. */
int amx_expert_cost(amx_ctx* ctx, const float* phi_e_rows, int ldphi, const float* w, int F, int n,
                    float c_min, float c_max, double* out, float* mean_out, double lambda_b,
                    void* stream);

/* The relabel's feature message (batch_reinforce.py:110-113 -> fit_cost's mean,
 * linear_cost.py:88): out[0..F) = the ordered fp64 column sums of n_parts rows of RFF
 * partials (as amx_sum_partials), out[F] = count -- the one buffer the cross-rank all-reduce
 * sums and amx_mmd_relabel reads. */
int amx_feature_message(amx_ctx* ctx, const double* partials, int n_parts, int F, double count,
                        double* out, void* stream);

/* The relabel tail in ONE launch (batch_reinforce.py:110-152 with linear_cost.py:84-109):
 * w = (float)(msg[f] / count) - phi_e[f] and mmd[0] = w.w exactly as amx_mmd_fit (count 0:
 * read msg[F]); the per-sample pessimistic reward of rows [0, n) of phi exactly as
 * amx_mmd_reward (clamp = 1: cost_range (c_min, c_max)) or amx_mmd_reward_raw (clamp = 0);
 * and, when expert_rows is given (clamp only), the expert cost exactly as amx_expert_cost
 * (expert_out: 1 + 1024 doubles, expert_mean: (1 - lambda_b) * mean in fp32).  `counter` is
 * one uint32 of device memory, zero before the first launch; the kernel leaves it zero.
 * One launch at a time per counter. */
int amx_mmd_relabel(amx_ctx* ctx, const double* msg, double count, const float* phi_e, int F,
                    float* w, float* mmd, const float* phi, int ldphi, const float* disc, float thr,
                    double lambda_b, int clamp, float c_min, float c_max, float* reward, float* ipm,
                    float* wbonus, int n, const float* expert_rows, int ld_e, int n_e,
                    double* expert_out, float* expert_mean, uint32_t* counter, void* stream);

/* ---- AMP / GAIL least-squares discriminator reward ---------------------------- */

/* Last Discriminator layer (512->1, milo/milo/gail_cost.py:18-42) fused with
 * get_ls_costs (:231-236) and get_bonus_costs (:254-279):
 *   D = h[n].w3 + b3; r = max(0, 1 - 0.25*(1-D)^2); ipm = (1-lambda)*(-r);
 *   bonus = lambda*disc[n] (raw disagreement); reward = -(ipm - bonus).
 * disc NULL -> plain get_costs path: reward = r. logits (nullable) receives D. */
int amx_amp_reward(amx_ctx* ctx, const float* h, int ldh, int Hd, const float* w3, float b3,
                   const float* disc, double lambda_b, float* reward, float* logits, int n,
                   void* stream);

/* amx_amp_reward for either discriminator loss type (GAILCost.get_costs,
 * gail_cost.py:246-251): AMX_DISC_LEAST_SQUARES as above, AMX_DISC_LOG_LIKELIHOOD
 * with input cost logsigmoid(D) (get_ll_costs, :238-244), r = -logsigmoid(D). */
int amx_disc_reward(amx_ctx* ctx, int loss_type, const float* h, int ldh, int Hd, const float* w3, float b3,
                    const float* disc, double lambda_b, float* reward, float* logits, int n, void* stream);

/* Cost-input rows of the non-'ss' input types ('sa', 'sas', 's', or AMP features):
 * out[b] = float32 [x0[b,:w0], x1[b,:w1], x2[b,:w2], 0...] up to ldc, fp64 sources
 * (linear_cost.py:115-127, gail_cost.py:258-268, batch_reinforce.py:107-110).
 * A segment with width 0 is absent (its pointer may be NULL). */
int amx_cost_rows(amx_ctx* ctx, const double* x0, long long ld0, int w0, const double* x1, long long ld1, int w1,
                  const double* x2, long long ld2, int w2, int B, float* out, int ldc, void* stream);

/* ---- returns / value baseline / GAE (the sampler's consumer) ------------------ */

/* Trajectory layout shared by the calls below ("segment grid"): L lanes of up to T
 * rows.  Lane l owns rows r(t, l) = base[l] + t * stride for t < len[l] (base NULL ->
 * base[l] = l; len NULL -> T).  end[r] closes a trajectory at row r: 0 = continues,
 * 1 = terminated (bootstrap 0), 2 = ends without termination (bootstrap with the
 * row's own baseline, mjrl's non-terminated rule); a lane's last row with end 0 is
 * treated as 2.  t0[l] (NULL -> 0) is the position of the lane's first row inside its
 * trajectory.  Engine buffers: base NULL, stride = lanes, end = done flags;
 * concatenated mjrl paths: base = path offsets, stride = 1, end = 1/2 at path ends. */

/* MLPBaseline._features (mjrl/mjrl/baselines/mlp_baseline.py:36-59): row r of feat
 * [.., ldf] f32 = [clip(obs[r], -10, 10) / 10, (tpos/1000)^1..4, 0 ...] computed in
 * fp64 and rounded to f32 (featmat.astype('float32'), :100); tpos = row position in
 * its trajectory.  Columns [S + 4, kf) are zeroed, kf = round_up(S + 4, 32). */
int amx_value_features(amx_ctx* ctx, int T, int L, const int32_t* len, const int32_t* t0,
                       const int64_t* base, long long stride, const uint8_t* end,
                       const double* obs, int ldo, float* feat, int ldf, void* stream);

/* Last Linear(H -> 1) of the MLPBaseline model (mlp_baseline.py:20-27, predict :99-108):
 * v[r] = b[0] + sum_k h[r][k] * w[k] (f32) for r < rows; H a multiple of 4. */
int amx_value_head(amx_ctx* ctx, int rows, const float* h, int ldh, int H, const float* w,
                   const float* b, float* v, void* stream);

/* compute_returns + compute_advantages (mjrl/mjrl/utils/process_samples.py:3-45):
 * per trajectory, in fp64 (numpy 1.21 promotion of the pinned reference env):
 *   ret[t] = rew[t] + gamma * ret[t+1]                            (discount_sum)
 *   GAE (gamma_lambda >= 0): delta[t] = (rew[t] + gamma * b1[t+1]) - b[t],
 *        adv[t] = delta[t] + gamma_lambda * adv[t+1]; b1 = b + [0 | b[-1]] at the end;
 *        delta is float64 for terminated trajectories and float32 arithmetic otherwise
 *        (np.append keeps b1 float32 when the appended value is b[-1])
 *   standard (gamma_lambda < 0): adv[t] = ret[t] - b[t].
 * rew (f32) is read at rbase[l] + t * rstride (rbase NULL -> l); v, ret, adv use r(t, l).
 * gamma_lambda = gamma * gae_lambda formed by the caller in double. */
int amx_gae(amx_ctx* ctx, int T, int L, const int32_t* len, const int64_t* base, long long stride,
            const uint8_t* end, const float* rew, const int64_t* rbase, long long rstride,
            const float* v, double gamma, double gamma_lambda, double* ret, double* adv,
            void* stream);

/* Advantage whitening of BatchREINFORCE.process_paths (mjrl/mjrl/algos/batch_reinforce.py:
 * 280-285): over the grid's rows, out = (adv - mean) / (std + eps) (population std);
 * stats[0..1] = mean, std (fp64, fixed reduction order).  out may alias adv.  Two launches over
 * the chip (per-block count / sum / M2, then the combine in block order and the apply); the
 * per-block partials live in the context (graph-capturable), so a context runs one whitening
 * at a time: do not issue two on different streams, or a captured one beside an eager one. */
int amx_adv_whiten(amx_ctx* ctx, int T, int L, const int32_t* len, const int64_t* base,
                   long long stride, const double* adv, double eps, double* out, double* stats,
                   void* stream);

/* ---- RNG ----------------------------------------------------------------------- */

/* Philox4x32-10 block for (key = seed, counter = {ctr0, ctr1, ctr2, ctr3}), written
 * to out[4*i .. 4*i+3] for i < n with ctr0 += i.  Exposed for parity tests of the
 * device RNG the reset/policy kernels use. */
int amx_philox(amx_ctx* ctx, uint64_t seed, uint32_t ctr1, uint32_t ctr2, uint32_t ctr3,
               uint32_t* out, int n, void* stream);

/* Host-side (no device, no context) policy noise of the reference sampler, bit-exact with
 * numpy's legacy RandomState as mjrl MLP.get_action draws it (mjrl/mjrl/policies/
 * gaussian_mlp.py:95-104: np.random.uniform() for the eps test, then np.random.randn(A), per
 * step) after get_samples' np.random.seed(seed) (milo/milo/sampler.py:39).  `states` is host
 * memory of n_states * AMX_MT_STATE_BYTES; amx_mt_seed seeds states[slots[i]] with seeds[i]
 * (np.random.seed(int)); amx_mt_policy_noise advances states[slots[i]] by `steps` get_action
 * calls, writing the randn values to out[k * ld_step + slots[i] * ld_slot + a] (doubles). */
int amx_mt_seed(void* states, int n_states, const int32_t* slots, const uint32_t* seeds, int n);
int amx_mt_policy_noise(void* states, int n_states, const int32_t* slots, int n, int steps, int A,
                        double* out, long long ld_step, long long ld_slot);

#ifdef __cplusplus
}
#endif
#endif /* AMX_HIP_H */
