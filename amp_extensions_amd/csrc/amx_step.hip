// Per-lane kernels of the batched SimEnv step (gym-simenv/gym_simenv/envs/sim_env.py):
// state assembly, fp64 state update + fall/horizon termination + ensemble disagreement,
// masked resets from a device reset-state table, and the device Gaussian-MLP policy.
//
// These kernels are HBM/latency-bound per lane row (a few KB per lane); the layout is one
// wave64 per lane with lanes of the wave striding the state vector, so every row access
// is coalesced and every per-lane reduction is a wave reduction (no LDS).
//
// Numerics: the file is built with -ffp-contract=off.  Every expression below that the
// reference evaluates as separate IEEE operations (normalisation, state update,
// termination sums/products) must round exactly as numpy/torch-CPU do; termination is
// bit-exact by construction.
#include "amx_common.h"

#include <utility>
#include <stdlib.h>

namespace {

// fp64 DPP move of both halves (lanes outside row_mask keep 0.0)
template <int CTRL, int RM>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, RM, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, RM, 0xf, false);
  return __hiloint2double(hi, lo);
}

// Sum over the wave's 64 lanes, returned to every lane, on the DPP path (no LDS): xor 1 and 2
// (quad_perm), the 8- and 16-lane mirrors (every lane of a row then holds the row sum), row
// 0 -> 1 and 2 -> 3 (row_bcast:15), rows 0+1 -> 2, 3 (row_bcast:31), lane 63 read back.  A fixed
// association: every caller (the fused step, k_disagreement) gets the same bits for the same
// lane values.  (The LDS-based __shfl_xor butterfly cost 5.7 us of the 8192-lane step kernel's
// 21.4 for its six pair sums, tools/step_time.py.)
__device__ inline double wave_sum(double v) {
  v += dpp_f64<0xb1, 0xf>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4e, 0xf>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141, 0xf>(v);  // row_half_mirror
  v += dpp_f64<0x140, 0xf>(v);  // row_mirror
  v += dpp_f64<0x142, 0xa>(v);  // row_bcast:15 into rows 1, 3
  v += dpp_f64<0x143, 0xc>(v);  // row_bcast:31 into rows 2, 3
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), 63);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), 63);
  return __hiloint2double(hi, lo);
}

// ---- assemble -----------------------------------------------------------------------
// x0 = [(s - mu_s)/sd_s, (a - mu_a)/sd_a, 0...] into every model's activation row.
// One wave per lane row; writes k0_pad columns for each of M models (once when stride_m is 0:
// the f16x3 GEMMs then read every model's x0 slice from model 0's rows).  With row_exp (the
// f16x3 GEMM's row-exponent slots, amx_row_exponents' layout) it also writes slot 0 = the
// exponent of the row's max |x0| and resets slots 1..n_slots-1 for every model.
template <typename T>
__global__ __launch_bounds__(256) void k_assemble(const T* __restrict__ ob, const T* __restrict__ act,
                                                  const float* __restrict__ norm, float* __restrict__ buf,
                                                  long long stride_m, int ldk, int S, int A, int M, int k0_pad,
                                                  int B, int* __restrict__ row_exp, long long stride_rexp,
                                                  long long slot_stride, int n_slots) {
  const int b = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const float* mu_s = norm;
  const float* sd_s = norm + S;
  const float* mu_a = norm + 2 * S;
  const float* sd_a = norm + 2 * S + A;
  uint32_t mx = 0;
  const int copies = stride_m == 0 ? 1 : M;  // stride 0: the models share one x0 slice
  for (int j = lane; j < k0_pad; j += 64) {
    float x = 0.f;
    if (j < S) {
      const float s = (float)ob[(long long)b * S + j];
      x = (s - mu_s[j]) / sd_s[j];
    } else if (j < S + A) {
      const int k = j - S;
      const float v = (float)act[(long long)b * A + k];
      x = (v - mu_a[k]) / sd_a[k];
    }
    for (int m = 0; m < copies; ++m) buf[m * stride_m + (long long)b * ldk + j] = x;
    const uint32_t bits = __float_as_uint(x) & 0x7fffffffu;
    mx = mx > bits ? mx : bits;
  }
  if (row_exp == nullptr) return;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t o = (uint32_t)__shfl_xor((int)mx, off);
    mx = mx > o ? mx : o;
  }
  if (lane < n_slots) {
    int e = (int)(mx >> 23) - 126;  // max|x0| < 2^e, clamped as the GEMM's exponents
    e = e < -100 ? -100 : (e > 100 ? 100 : e);
    const int v = lane == 0 ? e : -100;
    if (slot_stride < B) {  // member-blocked layout: row b % Bq of member block b / Bq, once
      const int Bq = (int)slot_stride, g = b / Bq;
      row_exp[g * stride_rexp + lane * slot_stride + (b - g * Bq)] = v;
    } else {
      for (int m = 0; m < M; ++m) row_exp[m * stride_rexp + lane * slot_stride + b] = v;
    }
  }
}

// ---- disagreement ---------------------------------------------------------------------
// d = max over pairs (i<j) of ||p_i - p_j||_2: the pair differences are formed in fp32 as
// torch does (preds[i] - preds[j]), squared and summed in fp64, sqrt in fp64, rounded.
template <int MM>
__device__ inline float lane_disagreement(const float* __restrict__ preds, long long strideP, int ldp, int b,
                                          int S, int lane) {
  constexpr int NP = MM * (MM - 1) / 2;
  double acc[NP > 0 ? NP : 1];
#pragma unroll
  for (int p = 0; p < (NP > 0 ? NP : 1); ++p) acc[p] = 0.0;
  for (int j = lane; j < S; j += 64) {
    float v[MM];
#pragma unroll
    for (int m = 0; m < MM; ++m) v[m] = preds[m * strideP + (long long)b * ldp + j];
    int p = 0;
#pragma unroll
    for (int i = 0; i < MM; ++i)
#pragma unroll
      for (int k = i + 1; k < MM; ++k) {
        const float d = v[i] - v[k];
        acc[p++] += (double)d * (double)d;
      }
  }
  // max over pairs of (float)sqrt(sum) == (float)sqrt(max over pairs of sum): sqrt and the
  // rounding are monotone, and the first-wins / NaN-skipping selection is the same on the sums
  double best = 0.0;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const double n = wave_sum(acc[p]);
    best = (p == 0 || n > best) ? n : best;
  }
  return (float)sqrt(best);
}

// Generic member count: one pair at a time (re-reads the L2-hot rows), few registers.
__device__ inline float lane_disagreement_any(const float* __restrict__ preds, long long strideP, int ldp, int b,
                                              int S, int M, int lane) {
  double best = 0.0;  // max of the sums, one sqrt (as lane_disagreement)
  bool first = true;
  for (int i = 0; i < M; ++i)
    for (int k = i + 1; k < M; ++k) {
      double acc = 0.0;
      for (int j = lane; j < S; j += 64) {
        const float d = preds[i * strideP + (long long)b * ldp + j] - preds[k * strideP + (long long)b * ldp + j];
        acc += (double)d * (double)d;
      }
      const double n = wave_sum(acc);
      best = (first || n > best) ? n : best;
      first = false;
    }
  return (float)sqrt(best);
}

// M = 4 (the MILO ensemble) gets the fused 6-pair pass; other sizes the generic loop.
// (A switch over every M would size the register file for M = 8 in every caller.)
__device__ inline float disagreement_dispatch(int M, const float* preds, long long strideP, int ldp, int b, int S,
                                              int lane) {
  if (M == 4) return lane_disagreement<4>(preds, strideP, ldp, b, S, lane);
  return M >= 2 ? lane_disagreement_any(preds, strideP, ldp, b, S, M, lane) : 0.f;
}

__global__ __launch_bounds__(256) void k_disagreement(const float* __restrict__ preds, long long strideP, int ldp,
                                                      float* __restrict__ disc, int S, int M, int B) {
  const int b = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const float d = disagreement_dispatch(M, preds, strideP, ldp, b, S, lane);
  if (lane == 0) disc[b] = d;
}

// ---- step + termination -----------------------------------------------------------------
struct StepArgs {
  const float* preds; long long strideP; int ldp;
  const int32_t* model_idx; int32_t* model_idx_out;  // (model_idx_out: fused reset only)
  const double* ob; double* ob_next;
  int32_t* num_steps; uint8_t* done; float* disc;
  float* cost_in; int ldc;
  int* cost_rexp;  // nullable: exponent of each cost row's max |x| (f16x3 RFF GEMM's row_exp)
  uint8_t* nonfinite;
  int S, M, B;
  amx_termination term;
  // fused reset (amx_step_reset; ob_out null = amx_step): done lanes restart from a table row
  // exactly as amx_reset_lanes(mask = done), the others copy ob' from registers
  double* ob_out; const double* table; int R; const int32_t* rows; uint32_t k0, k1;
  int32_t* reset_count; int32_t* row_out;
  int32_t* steps0_out;  // nullable: num_steps before this step (a rollout's first slot)
  uint64_t* counter; long long counter_delta;  // nullable: *counter += delta (graph replays' policy counter)
  double* ob_rec;  // nullable: a copy of ob (a rollout's slot 0 when the carried state is read in place)
};

// NIT = ceil(S/64) state elements per lane, kept in registers: all loads of the row are
// issued up front, and the fall check reads the few values it needs from the owning lanes
// with shuffles instead of re-loading them (the kernel is latency-bound, not HBM-bound).
// MM4: the MILO ensemble (M = 4): all four members' rows are loaded in the first phase and
// the disagreement is formed from registers (one memory round trip instead of two; the same
// per-lane j order as lane_disagreement, so the same bits).
// srow (nullable, LDS): the float32 of the lane's next observation obs[t+1] (ob', or its reset
// row), written lane-distinctly -- the input row of the fused policy (k_step_act)
template <int NIT, bool MM4>
__device__ __forceinline__ void step_lane(const StepArgs& a, int b, int lane, float* srow) {
  const amx_termination& T = a.term;
  const int S = a.S;
  const int k = a.model_idx[b];
  // the lane's counters (and the caller's reset row) are loaded with the row, not after the
  // row's stores the compiler cannot move them above (round 3: within noise at 8192 / 5120
  // lanes, profiles/r03e_step_ab.txt -- the later loads were already overlapped by other waves)
  const int ns0 = a.num_steps[b];
  const int rc0 = a.ob_out ? a.reset_count[b] : 0;
  const int row0 = (a.ob_out && a.rows) ? a.rows[b] : 0;
  const double* ob = a.ob + (long long)b * S;
  double* on = a.ob_next + (long long)b * S;

  double o[NIT], x[NIT];
  float p[NIT];
  float pm[MM4 ? 4 : 1][NIT];
  if constexpr (MM4) {
    const float* pb = a.preds + (long long)b * a.ldp;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int j = lane + 64 * it;
      o[it] = j < S ? ob[j] : 0.0;
#pragma unroll
      for (int m = 0; m < 4; ++m) pm[m][it] = j < S ? pb[m * a.strideP + j] : 0.f;
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it)
      p[it] = k == 0 ? pm[0][it] : k == 1 ? pm[1][it] : k == 2 ? pm[2][it] : pm[3][it];
  } else {
    const float* pk = a.preds + (long long)k * a.strideP + (long long)b * a.ldp;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int j = lane + 64 * it;
      o[it] = j < S ? ob[j] : 0.0;
      p[it] = j < S ? pk[j] : 0.f;
    }
  }
  // sim_env.py:158  ob += state_diff (float32 -> float64), then the in-place velocity
  // rescale of check_velocity (:264-267) when RecordVelAsPos and the check are enabled.
  const bool vscale = T.vel_check && T.record_vel_as_pos;
  bool vel_bad = false, bad = false;
  uint32_t cmax = 0;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int j = lane + 64 * it;
    double v = o[it] + (double)p[it];
    if (vscale && j >= T.vel_offset) v = v / T.sampling_rate;
    x[it] = v;
    if (j < S) {
      on[j] = v;
      if (a.ob_rec) a.ob_rec[(long long)b * S + j] = o[it];
      if (T.vel_check && j >= T.vel_offset) vel_bad |= fabs(v) > T.vel_thresh;
      bad |= !isfinite(v);
      if (a.cost_in) {
        const float c0 = (float)o[it], c1 = (float)v;
        a.cost_in[(long long)b * a.ldc + j] = c0;
        a.cost_in[(long long)b * a.ldc + S + j] = c1;
        const uint32_t u0 = __float_as_uint(c0) & 0x7fffffffu, u1 = __float_as_uint(c1) & 0x7fffffffu;
        cmax = cmax > u0 ? cmax : u0;
        cmax = cmax > u1 ? cmax : u1;
      }
    }
  }
  if (a.cost_in) {  // zero the K padding of the cost-input row
    for (int j = 2 * S + lane; j < a.ldc; j += 64) a.cost_in[(long long)b * a.ldc + j] = 0.f;
    if (a.cost_rexp) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        const uint32_t oo = (uint32_t)__shfl_xor((int)cmax, off);
        cmax = cmax > oo ? cmax : oo;
      }
      if (lane == 0) {
        int e = (int)(cmax >> 23) - 126;  // max|row| < 2^e (amx_row_exponents' clamp)
        a.cost_rexp[b] = e < -100 ? -100 : (e > 100 ? 100 : e);
      }
    }
  }

  // fall check (sim_env.py:175-257): lane i < n evaluates body i; every lane takes part
  // in the shuffles that fetch ob'[j] from the lane that owns element j.
  auto fetch = [&](int j) -> double {
    const int src = j & 63, itj = j >> 6;
    double r = 0.0;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const double v = __shfl(x[it], src);
      r = (itj == it) ? v : r;
    }
    return r;
  };
  const int bi = lane < T.n ? lane : 0;
  const double root_y = fetch(0);
  const double rel_y = fetch(T.y_index[bi]);
  const double ny = fetch(T.shape[bi] == AMX_SHAPE_CAPSULE ? T.ny_index[bi] : 0);
  bool hit = false;
  if (lane < T.n && (T.shape[bi] == AMX_SHAPE_SPHERE || T.shape[bi] == AMX_SHAPE_CAPSULE)) {
    const double y = T.list_index_world[bi] ? rel_y : root_y + rel_y;
    if (T.shape[bi] == AMX_SHAPE_SPHERE) {
      hit = y <= T.thresh[bi];
    } else {
      const double top = T.half_h[bi] * ny;
      const double bot = T.neg_half_h[bi] * ny;
      const double ytop = y + top;
      const double ybot = y + bot;
      hit = (ytop <= T.thresh[bi]) || (ybot <= T.thresh[bi]);
    }
  }  // box: check_box always False (sim_env.py:238-244)
  const bool collided = __ballot(hit) != 0ull;
  const bool vexp = __ballot(vel_bad) != 0ull;
  const bool nf = __ballot(bad) != 0ull;

  float d = 0.f;
  if constexpr (MM4) {
    if (a.disc) {
      double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        if (lane + 64 * it < S) {
          int q = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int kk = i + 1; kk < 4; ++kk) {
              const float df = pm[i][it] - pm[kk][it];
              acc[q++] += (double)df * (double)df;
            }
        }
      }
      double mx = 0.0;  // one sqrt of the max sum (lane_disagreement)
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        const double n = wave_sum(acc[q]);
        mx = (q == 0 || n > mx) ? n : mx;
      }
      d = (float)sqrt(mx);
    }
  } else {
    if (a.disc) d = disagreement_dispatch(a.M, a.preds, a.strideP, a.ldp, b, S, lane);
  }

  const int ns = ns0 + 1;  // sim_env.py:153
  const bool horizon_done = ns >= T.horizon;  // :170
  const bool dn = horizon_done || collided || vexp;  // wave-uniform
  bool reset = false;
  if (a.ob_out) {  // the next step's observation (amx_reset_lanes with mask = done)
    double* oo = a.ob_out + (long long)b * S;
    if (!dn) {
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int j = lane + 64 * it;
        if (j < S) {
          oo[j] = x[it];
          if (srow) srow[j] = (float)x[it];  // np.float32(observation)
        }
      }
      if (lane == 0 && a.row_out) a.row_out[b] = -1;
    } else {
      reset = true;
      const int rc = rc0 + 1;  // sim_env.py:282
      int row;
      if (a.rows) {
        row = row0;
      } else {
        const amx::u32x4 r = amx::philox4x32_10({(uint32_t)b, (uint32_t)rc, 0u, amx::kTagReset}, a.k0, a.k1);
        row = (int)((((uint64_t)r.y << 32) | r.x) % (uint64_t)a.R);
      }
      const double* src = a.table + (long long)row * S;
      for (int j = lane; j < S; j += 64) {
        const double v = src[j];
        oo[j] = v;
        if (srow) srow[j] = (float)v;
      }
      if (lane == 0) {
        a.reset_count[b] = rc;
        a.model_idx_out[b] = rc % a.M;  // :282-283
        if (a.row_out) a.row_out[b] = row;
      }
    }
  }

  if (a.counter && b == 0 && lane == 0) a.counter[0] += (uint64_t)a.counter_delta;  // amx_counter_add
  if (lane == 0) {
    if (a.steps0_out) a.steps0_out[b] = ns - 1;
    a.num_steps[b] = reset ? 0 : ns;  // a reset restarts the episode counter (:277)
    a.done[b] = dn ? 1 : 0;
    if (a.disc) a.disc[b] = d;
    if (a.nonfinite) a.nonfinite[b] = nf ? 1 : 0;
  }
}

template <int NIT, bool MM4>
__global__ __launch_bounds__(256) void k_step(StepArgs a) {
  const int b = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (b >= a.B) return;  // wave-uniform
  step_lane<NIT, MM4>(a, b, lane, nullptr);
}

// ---- reset ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_reset(const uint8_t* __restrict__ mask, const double* __restrict__ table,
                                               int R, const int32_t* __restrict__ rows, uint32_t k0, uint32_t k1,
                                               const double* ob_src, double* ob_out, int32_t* num_steps,
                                               int32_t* model_idx, int32_t* reset_count, int32_t* row_out, int S,
                                               int M, int B) {
  const int b = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const bool do_reset = (mask == nullptr) || mask[b] != 0;
  if (!do_reset) {
    if (ob_src != ob_out)
      for (int j = lane; j < S; j += 64) ob_out[(long long)b * S + j] = ob_src[(long long)b * S + j];
    if (lane == 0 && row_out) row_out[b] = -1;
    return;
  }
  const int rc = reset_count[b] + 1;  // sim_env.py:282: counter advances on every reset
  int row;
  if (rows) {
    row = rows[b];
  } else {
    const amx::u32x4 r = amx::philox4x32_10({(uint32_t)b, (uint32_t)rc, 0u, amx::kTagReset}, k0, k1);
    const uint64_t x = ((uint64_t)r.y << 32) | r.x;
    row = (int)(x % (uint64_t)R);
  }
  const double* src = table + (long long)row * S;
  for (int j = lane; j < S; j += 64) ob_out[(long long)b * S + j] = src[j];
  if (lane == 0) {
    reset_count[b] = rc;
    model_idx[b] = rc % M;  // :282-283
    num_steps[b] = 0;       // :277
    if (row_out) row_out[b] = row;
  }
}

// ---- policy ----------------------------------------------------------------------------------
// One workgroup = 256 threads (4 waves) serving 16 lanes.  The whole MLP (W1 [H1][S], W2, W3)
// and the lanes' float32 observations are staged in LDS once per workgroup; every dense layer
// runs on the matrix pipe (v_mfma_f32_16x16x4_f32: the 16 lanes are the M dimension), its
// 16-unit column blocks (and, for narrow layers, K halves) dealt over the 4 waves, then one
// combine pass applies the fixed-order K-part sum, the bias and tanh.  Every LDS fragment read
// is lane-distinct (no broadcast reads: see the note at pol_mfma_layer).  The Gaussian noise
// takes one Philox block and one Box-Muller per (lane, action pair): both normals of the pair.
constexpr int POL_LANES = 16;
constexpr int POL_MAXH = 256;
constexpr int POL_X0_COLS = 320;  // fused assembly: k0_pad (= S + A rounded up to 32) at most this

__host__ __device__ inline int pol_stride(int k) {  // row stride (floats) for a [*, k] LDS matrix
  const int r = (k + 3) & ~3;
  return (r % 8 == 0) ? r + 4 : r;
}

// Packed weight image (amx_policy_pack): [W1 H1 x s1 | W2 H2 x s2 | W3 A x s3 | b1 | b2 | b3],
// zero-padded rows, total rounded to whole float4s.  The action kernel copies it into LDS
// as is.
__host__ __device__ inline int pol_blob_floats(int S, int H1, int H2, int A) {
  const int s1 = pol_stride(S), s2 = pol_stride(H1), s3 = pol_stride(H2);
  return (H1 * s1 + H2 * s2 + A * s3 + H1 + H2 + A + 3) & ~3;
}

// floats of the layers' partial-sum area: K parts x 16 lanes x (16 x column blocks)
__host__ __device__ inline int pol_part_floats(int H1, int H2, int A) {
  int h = H1 > H2 ? H1 : H2;
  h = h > A ? h : A;
  const int w = 16 * ((h + 15) / 16);
  return POL_LANES * (w > 64 ? w : 64);
}

__host__ inline size_t pol_lds_bytes(int S, int H1, int H2, int A) {
  const int s1 = pol_stride(S), s2 = pol_stride(H1), s3 = pol_stride(H2);
  const size_t fl = (size_t)pol_blob_floats(S, H1, H2, A) + POL_LANES * (s1 + s2 + s3 + 2 * A) +
                    pol_part_floats(H1, H2, A);
  return fl * sizeof(float);
}

struct PolicyArgs {
  const double* ob; const float* blob; int H1; int H2; const double* nscale; const double* noise;
  uint32_t k0, k1, ctr_lo, ctr_hi; int eval_mode;
  const uint64_t* ctr_dev;  // nullable: the counter read from device memory (graph replays)
  double* act; float* mean_out;
  float* x0; long long stride_m; int ldk; int k0_pad; int M; const float* norm;
  int* row_exp; long long stride_rexp; long long slot_stride; int n_slots;  // nullable (k_assemble's)
  int S, A, B;
};

typedef float pf4 __attribute__((ext_vector_type(4)));

constexpr int POL_STAGE_W = 12;  // float4 loads of the weight image per thread per pass
constexpr int POL_STAGE_O = 16;  // double loads of observations per thread per pass

// zero the pad columns [cols, ds) of rows [0, rows)
__device__ inline void pol_zero_pads(float* __restrict__ dst, int ds, int cols, int rows) {
  const int w = ds - cols;
  for (int i = threadIdx.x; i < rows * w; i += 256) dst[(i / w) * ds + cols + i % w] = 0.f;
}

// One pass issues every global load (weight image float4s, observation doubles) before
// any LDS store: the staging costs one memory round trip instead of one per array.
__device__ inline void pol_stage_all(float* __restrict__ img, const float* __restrict__ blob, int n4,
                                     float* __restrict__ so, int s1, const double* __restrict__ ob, int n_ob,
                                     int S) {
  const int t = threadIdx.x;
  for (int it = 0;; ++it) {
    const int w0 = t + it * 256 * POL_STAGE_W, o0 = t + it * 256 * POL_STAGE_O;
    if (w0 >= n4 && o0 >= n_ob) break;
    pf4 wv[POL_STAGE_W];
    double ov[POL_STAGE_O];
#pragma unroll
    for (int u = 0; u < POL_STAGE_W; ++u) {
      const int i = w0 + u * 256;
      if (i < n4) wv[u] = reinterpret_cast<const pf4*>(blob)[i];
    }
#pragma unroll
    for (int u = 0; u < POL_STAGE_O; ++u) {
      const int i = o0 + u * 256;
      if (i < n_ob) ov[u] = ob[i];
    }
#pragma unroll
    for (int u = 0; u < POL_STAGE_W; ++u) {
      const int i = w0 + u * 256;
      if (i < n4) reinterpret_cast<pf4*>(img)[i] = wv[u];
    }
#pragma unroll
    for (int u = 0; u < POL_STAGE_O; ++u) {
      const int i = o0 + u * 256;
      if (i < n_ob) {
        const int r = i / S, c = i - r * S;
        so[r * s1 + c] = (float)ov[u];  // np.float32(observation)
      }
    }
  }
}

// One dense layer of the workgroup's 16 lanes on the matrix pipe: the raw x . W^T of 16 lanes x
// N units, x rows [16][ldx] and W rows [N][ldw] in LDS, zero beyond K up to 4 nc.  Column block
// nb (16 units) and K part kh of nblk x ksplit work items per wave (wave w takes items w, w + 4,
// ...): 16x16x4 MFMAs over the chunks c = kq + 4 jj of its part, lane (i = l & 15, kq = l >> 4)
// reading one float4 of x row i and one of W row 16 nb + i per 4 MFMAs (k = 4c + e: a
// permutation of the K order, as any blocked fp32 matmul).  Fragment reads are lane-distinct:
// a broadcast ds_read_b128 (all 16 threads of a row reading the same 16 B) returned wrong data
// in lanes 48-63 on gfx950 beside a co-resident 16x16x32 f16 MFMA workgroup (tools/victim.hip
// + tools/corunner.hip).  The raw partials go to `part` [ksplit][16][16 nblk]; after a barrier
// pol_combine sums the K parts in order.  (Round 2: 3 MFMA layers + combine passes took the
// in-kernel time from 17.4 to 15.9 us at 8192 lanes; the DPP-broadcast FMA chains before
// spent 4.5 us in layer 1 alone.)
__device__ inline int pol_ksplit(int nblk, int nc) {
  const int jjt = (nc + 3) >> 2;
  return nblk >= 4 ? 1 : (4 / nblk < jjt ? 4 / nblk : jjt);
}

__device__ inline void pol_mfma_layer(const float* __restrict__ x, int ldx, int nc, const float* __restrict__ w,
                                      int ldw, int N, float* __restrict__ part) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, kq = lane >> 4;
  const int nblk = (N + 15) >> 4, jjt = (nc + 3) >> 2, ksplit = pol_ksplit(nblk, nc);
  const int ldp = 16 * nblk;
  for (int item = wave; item < nblk * ksplit; item += 4) {
    const int nb = item % nblk, kh = item / nblk;
    const int jj0 = kh * jjt / ksplit, jj1 = (kh + 1) * jjt / ksplit;
    const int u = 16 * nb + i;
    const float* xr = x + i * ldx;
    const float* wr = w + (u < N ? u : 0) * ldw;
    pf4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int jj = jj0; jj < jj1; ++jj) {
      const int c = kq + 4 * jj;
      const bool ok = c < nc;
      const pf4 a = ok ? *reinterpret_cast<const pf4*>(xr + 4 * c) : pf4{0.f, 0.f, 0.f, 0.f};
      const pf4 b = (ok && u < N) ? *reinterpret_cast<const pf4*>(wr + 4 * c) : pf4{0.f, 0.f, 0.f, 0.f};
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
    }
    float* pp = part + kh * 16 * ldp + 16 * nb + i;  // D row 4 kq + r, column i
#pragma unroll
    for (int r = 0; r < 4; ++r) pp[(4 * kq + r) * ldp] = acc[r];
  }
}

// out[l][u] = act(sum over K parts + bias) for the 16 lanes x N units (after a barrier)
__device__ inline void pol_combine(const float* __restrict__ part, int N, int nc, const float* __restrict__ bias,
                                   bool tanh_act, float* __restrict__ out, int ldo) {
  const int nblk = (N + 15) >> 4, ksplit = pol_ksplit(nblk, nc), ldp = 16 * nblk;
  for (int e = threadIdx.x; e < POL_LANES * N; e += 256) {
    const int l = e / N, u = e - l * N;
    float z = part[l * ldp + u];
    for (int kh = 1; kh < ksplit; ++kh) z += part[(kh * 16 + l) * ldp + u];
    z = z + bias[u];                               // nn.Linear: x W^T + b
    out[l * ldo + u] = tanh_act ? tanhf(z) : z;    // FCNetwork: tanh hidden, identity output
  }
}

// The policy of one workgroup's 16 lanes once its LDS is staged (k_policy; k_step_act): the
// lanes' float32 observations in `so`, the weight image at psm.  Only threads < 256 (the first
// four waves) work: k_step_act's other twelve waves take part in the barriers only, so the work
// decomposition -- and every bit of the result -- is k_policy's.
__device__ __forceinline__ void policy_core(const PolicyArgs& p, float* psm, int b0, int img_floats) {
  const int S = p.S, A = p.A, H1 = p.H1, H2 = p.H2;
  const int s1 = pol_stride(S), s2 = pol_stride(H1), s3 = pol_stride(H2);
  float* w1 = psm;                       // [H1][s1]   (packed image, amx_policy_pack)
  float* w2 = w1 + H1 * s1;              // [H2][s2]
  float* w3 = w2 + H2 * s2;              // [A][s3]
  float* bb1 = w3 + A * s3;
  float* bb2 = bb1 + H1;
  float* bb3 = bb2 + H2;
  float* so = psm + img_floats;          // [16][s1] (after the weight image's LDS slot)
  float* h1 = so + POL_LANES * s1;       // [16][s2]
  float* h2 = h1 + POL_LANES * s2;       // [16][s3]
  float* mo = h2 + POL_LANES * s3;       // [16][A] policy means
  float* xa_s = mo + POL_LANES * A;      // [16][A] float32 actions for the fused assembly
  float* part = xa_s + POL_LANES * A;    // layer partial sums (pol_part_floats)
  const int t = threadIdx.x;
  const bool on = t < 256;               // wave-uniform
  const int nc1 = (S + 3) >> 2, nc2 = (H1 + 3) >> 2, nc3 = (H2 + 3) >> 2;
  // the injected noise and the noise scale of this thread's (lane, action pair) items, loaded
  // before the layers so the round trip hides under them (the action loop below: at most
  // POL_PRE items per thread)
  const int npairs = (A + 1) >> 1;
  constexpr int POL_PRE = 2;
  double pre_n[POL_PRE][2], pre_s[POL_PRE][2];
#pragma unroll
  for (int q = 0; q < POL_PRE; ++q) {
    const int e = t + 256 * q;
    const int l = e / npairs, pr = e - l * npairs, b = b0 + l;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int u = 2 * pr + h;
      const bool ok = on && e < POL_LANES * npairs && b < p.B && u < A;
      pre_n[q][h] = (ok && p.noise && !p.eval_mode) ? p.noise[(long long)b * A + u] : 0.0;
      pre_s[q][h] = (ok && !p.eval_mode) ? p.nscale[u] : 0.0;
    }
  }
  if (on) pol_mfma_layer(so, s1, nc1, w1, s1, H1, part);
  __syncthreads();
  if (on) pol_combine(part, H1, nc1, bb1, true, h1, s2);
  __syncthreads();
  if (on) pol_mfma_layer(h1, s2, nc2, w2, s2, H2, part);
  __syncthreads();
  if (on) pol_combine(part, H2, nc2, bb2, true, h2, s3);
  __syncthreads();
  if (on) pol_mfma_layer(h2, s3, nc3, w3, s3, A, part);
  __syncthreads();
  if (on) pol_combine(part, A, nc3, bb3, false, mo, A);  // FCNetwork out_scale = 1, out_shift = 0 (fc_network.py:54)
  __syncthreads();
  // actions: one thread per (lane, pair u = 2pr, 2pr + 1): Box-Muller on one Philox block gives
  // both normals of the pair (gaussian_mlp.py:102-103: float32 mean + float64 noise)
  uint32_t ctr_lo = p.ctr_lo, ctr_hi = p.ctr_hi;
  if (p.ctr_dev) {  // device counter + the by-value offset
    const uint64_t cv = *p.ctr_dev + ((uint64_t)p.ctr_hi << 32 | p.ctr_lo);
    ctr_lo = (uint32_t)cv;
    ctr_hi = (uint32_t)(cv >> 32);
  }
  // item e = (lane l, pair pr); items t and t + 256 use the prefetched noise, any further ones
  // (A > 2 * 256 / POL_LANES) load it here
  auto act_item = [&](int e, const double* pn, const double* ps) {
    const int l = e / npairs, pr = e - l * npairs;
    const int b = b0 + l;
    if (b >= p.B) return;
    double n[2] = {0.0, 0.0};
    if (!p.eval_mode && !p.noise) {
      const amx::u32x4 r = amx::philox4x32_10(
          {(uint32_t)b, ctr_lo, ((uint32_t)pr << 8) | (ctr_hi & 0xffu), amx::kTagPolicy}, p.k0, p.k1);
      const double u1 = 1.0 - amx::u53(r.x, r.y);  // (0, 1]
      const double u2 = amx::u53(r.z, r.w);
      const double rad = sqrt(-2.0 * log(u1));
      const double ang = 6.283185307179586 * u2;
      n[0] = rad * cos(ang);
      n[1] = rad * sin(ang);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int u = 2 * pr + h;
      if (u >= A) break;
      const float m = mo[l * A + u];
      if (p.mean_out) p.mean_out[(long long)b * A + u] = m;
      double a_out;
      if (p.eval_mode) {
        a_out = (double)m;
      } else {
        const double nz = p.noise ? (pn ? pn[h] : p.noise[(long long)b * A + u]) : n[h];
        a_out = (double)m + (ps ? ps[h] : p.nscale[u]) * nz;
      }
      p.act[(long long)b * A + u] = a_out;
      if (p.x0) xa_s[l * A + u] = (float)a_out;
    }
  };
  if (on) {
#pragma unroll
    for (int q = 0; q < POL_PRE; ++q)
      if (t + 256 * q < POL_LANES * npairs) act_item(t + 256 * q, pre_n[q], pre_s[q]);
    for (int e = t + 256 * POL_PRE; e < POL_LANES * npairs; e += 256) act_item(e, nullptr, nullptr);
  }
  if (!p.x0) return;
  __syncthreads();
  if (!on) return;  // (after the last barrier)
  // fused amx_assemble_input[_rexp] (dynamics.py:225-227): 16 threads per row (one DPP row of
  // the wave; columns c0 + 16q), the block's POL_LANES rows of x0 (once when stride_m is 0: the
  // f16x3 GEMMs read every model's x0 slice from model 0's rows, else for every model), and
  // with row_exp slot 0 = the exponent of the row's max |x0| and slots 1..n_slots-1 reset, for
  // every model -- the same values and bits as k_assemble
  const float* mu_s = p.norm;
  const float* sd_s = p.norm + S;
  const float* mu_a = p.norm + 2 * S;
  const float* sd_a = p.norm + 2 * S + A;
  const int k0 = p.k0_pad;
  const int copies = p.stride_m == 0 ? 1 : p.M;
  const int ll = t >> 4, c0 = t & 15;  // 256 threads = the 16 rows x 16 column lanes
  const int bb = b0 + ll;
  const bool row_ok = bb < p.B;
  // the normalizers of this thread's columns, loaded together (one round trip, not one per column)
  constexpr int QT = POL_X0_COLS / 16;
  float mu[QT], sd[QT];
#pragma unroll
  for (int q = 0; q < QT; ++q) {
    const int j = c0 + 16 * q;
    mu[q] = 0.f;
    sd[q] = 1.f;
    if (j < S) {
      mu[q] = mu_s[j];
      sd[q] = sd_s[j];
    } else if (j < S + A) {
      mu[q] = mu_a[j - S];
      sd[q] = sd_a[j - S];
    }
  }
  uint32_t mx = 0;
  if (row_ok) {
#pragma unroll
    for (int q = 0; q < QT; ++q) {
      const int j = c0 + 16 * q;
      if (j >= k0) break;
      float x = 0.f;
      if (j < S) {
        x = (so[ll * s1 + j] - mu[q]) / sd[q];
      } else if (j < S + A) {
        x = (xa_s[ll * A + j - S] - mu[q]) / sd[q];
      }
      for (int mm = 0; mm < copies; ++mm) p.x0[mm * p.stride_m + (long long)bb * p.ldk + j] = x;
      const uint32_t bits = __float_as_uint(x) & 0x7fffffffu;
      mx = mx > bits ? mx : bits;
    }
  }
  if (p.row_exp == nullptr) return;
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) {  // max over the row's 16 threads
    const uint32_t o = (uint32_t)__shfl_xor((int)mx, off);
    mx = mx > o ? mx : o;
  }
  if (!row_ok) return;
  int e = (int)(mx >> 23) - 126;  // max|x0| < 2^e, clamped as the GEMM's exponents
  e = e < -100 ? -100 : (e > 100 ? 100 : e);
  for (int sl = c0; sl < p.n_slots; sl += 16) {
    const int v = sl == 0 ? e : -100;
    if (p.slot_stride < p.B) {  // member-blocked layout (as k_assemble)
      const int Bq = (int)p.slot_stride, g = bb / Bq;
      p.row_exp[g * p.stride_rexp + sl * p.slot_stride + (bb - g * Bq)] = v;
    } else {
      for (int mm = 0; mm < p.M; ++mm) p.row_exp[mm * p.stride_rexp + sl * p.slot_stride + bb] = v;
    }
  }
}


__global__ __launch_bounds__(256) void k_policy(PolicyArgs p) {
  extern __shared__ __attribute__((aligned(16))) float psm[];
  const int S = p.S, s1 = pol_stride(S), s2 = pol_stride(p.H1), s3 = pol_stride(p.H2);
  const int nblob = pol_blob_floats(S, p.H1, p.H2, p.A);
  float* so = psm + nblob;               // [16][s1]
  float* h1 = so + POL_LANES * s1;       // [16][s2], then h2 [16][s3]
  const int t = threadIdx.x;
  const int b0 = blockIdx.x * POL_LANES;
  // staging: the packed weight image (pads already zero) and the block's observation rows;
  // the observation pads / rows of lanes >= B are zeroed (they take part in the MFMAs)
  const int nl = (p.B - b0) < POL_LANES ? (p.B - b0) : POL_LANES;  // valid lanes of this block
  pol_zero_pads(so, s1, S, nl);
  for (int i = t + nl * s1; i < POL_LANES * s1; i += 256) so[i] = 0.f;
  pol_stage_all(psm, p.blob, nblob >> 2, so, s1, p.ob + (long long)b0 * S, nl * S, S);
  for (int i = t; i < POL_LANES * (s2 + s3); i += 256) h1[i] = 0.f;  // pads of h1/h2
  __syncthreads();
  policy_core(p, psm, b0, nblob);
}

// ---- fused step + next action --------------------------------------------------------------
// One workgroup = 16 waves = the 16 lanes of one policy block: wave w runs step t of lane
// b0 + w (step_lane, amx_step_reset's fused form: update, termination, disagreement, cost row,
// table reset) and leaves the float32 of the lane's obs[t+1] in its LDS row, then the block
// runs the policy of step t + 1 on those rows (policy_core: actions, means, and the fused x0 +
// row-exponent assembly of step t + 1's ensemble forward) -- the same values and bits as
// amx_step_reset followed by amx_policy_act on obs[t+1], in one launch with the observation
// rows kept on chip.  The weight image arrives by LDS-DMA (global_load_lds, whole 1-KiB pieces:
// amx_policy_blob_floats rounds the image up to them) issued before the step's loads, so it is
// in flight under the step phase without holding registers.
__host__ __device__ inline int pol_image_lds_floats(int S, int H1, int H2, int A) {
  return (pol_blob_floats(S, H1, H2, A) + 255) & ~255;
}

// W8: two workgroups per CU (<= 64 VGPRs, 8 waves per SIMD) instead of one
template <int NIT, bool MM4, bool W8>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(W8 ? 8 : 1))) void k_step_act(StepArgs a,
                                                                                                    PolicyArgs p) {
  extern __shared__ __attribute__((aligned(16))) float psm[];
  const int S = p.S, s1 = pol_stride(S), s2 = pol_stride(p.H1), s3 = pol_stride(p.H2);
  const int nimg = pol_image_lds_floats(S, p.H1, p.H2, p.A);
  float* so = psm + nimg;                // [16][s1]
  float* h1 = so + POL_LANES * s1;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int b0 = blockIdx.x * POL_LANES, b = b0 + wave;
  for (int q = wave; q < (nimg >> 8); q += POL_LANES)  // 256 floats = one 1-KiB piece per wave-instruction
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p.blob + q * 256 + 4 * lane),
                                     (__attribute__((address_space(3))) void*)(psm + q * 256), 16, 0, 0);
  float* srow = so + wave * s1;
  if (b < a.B) {  // wave-uniform
    step_lane<NIT, MM4>(a, b, lane, srow);
    for (int j = S + lane; j < s1; j += 64) srow[j] = 0.f;
  } else {
    for (int j = lane; j < s1; j += 64) srow[j] = 0.f;
  }
  for (int i = t; i < POL_LANES * (s2 + s3); i += 1024) h1[i] = 0.f;  // pads of h1/h2
  __syncthreads();  // (waits for the image's DMA: vmcnt(0) before the barrier)
  policy_core(p, psm, b0, nimg);
}

// amx_policy_pack: nn.Linear weights -> the zero-padded LDS image (one thread per float).
__global__ void k_policy_pack(const float* __restrict__ W1, const float* __restrict__ b1, int H1,
                              const float* __restrict__ W2, const float* __restrict__ b2, int H2,
                              const float* __restrict__ W3, const float* __restrict__ b3, int S, int A,
                              float* __restrict__ blob) {
  const int s1 = pol_stride(S), s2 = pol_stride(H1), s3 = pol_stride(H2);
  const int n = pol_blob_floats(S, H1, H2, A);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int j = i;
  float v = 0.f;
  if (j < H1 * s1) {
    const int r = j / s1, c = j % s1;
    v = c < S ? W1[(long long)r * S + c] : 0.f;
  } else if ((j -= H1 * s1) < H2 * s2) {
    const int r = j / s2, c = j % s2;
    v = c < H1 ? W2[r * H1 + c] : 0.f;
  } else if ((j -= H2 * s2) < A * s3) {
    const int r = j / s3, c = j % s3;
    v = c < H2 ? W3[r * H2 + c] : 0.f;
  } else if ((j -= A * s3) < H1) {
    v = b1[j];
  } else if ((j -= H1) < H2) {
    v = b2[j];
  } else if ((j -= H2) < A) {
    v = b3[j];
  }
  blob[i] = v;
}

__global__ void k_philox(uint32_t k0, uint32_t k1, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const amx::u32x4 r = amx::philox4x32_10({(uint32_t)i, c1, c2, c3}, k0, k1);
  out[4 * i + 0] = r.x;
  out[4 * i + 1] = r.y;
  out[4 * i + 2] = r.z;
  out[4 * i + 3] = r.w;
}

inline dim3 lanes_grid(int B) { return dim3((unsigned)((B + 3) / 4)); }  // 4 lane-waves per block

}  // namespace

// the member-blocked row-exponent layout (slot_stride = Bq < B): B = M' x Bq lanes, M' <= M member
// blocks, x0 written once (stride_m 0), member block g's slots at g * stride_rexp
static bool blocked_rexp_ok(const amx_ctx* ctx, int B, long long stride_m, long long stride_rexp, long long slot_stride,
                            int n_slots) {
  return ctx && stride_m == 0 && slot_stride > 0 && B % slot_stride == 0 && B / slot_stride <= ctx->M &&
         stride_rexp >= (long long)n_slots * slot_stride;
}

static int assemble(const char* fn, amx_ctx* ctx, const void* ob, const void* act, int in_dtype, float* act_buf,
                    long long stride_m, int ldk, int B, int* row_exp, long long stride_rexp, long long slot_stride,
                    int n_slots, void* stream) {
  AMX_CHECK_ARG(ctx && ctx->have_norm, "%s: context has no normalizers", fn);
  AMX_CHECK_ARG(ob && act && act_buf, "%s: null pointer", fn);
  AMX_CHECK_ARG(B >= 0, "%s: B=%d", fn, B);
  AMX_CHECK_ARG(ldk >= ctx->k0_pad, "%s: ldk=%d < k0_pad=%d", fn, ldk, ctx->k0_pad);
  AMX_CHECK_ARG(ctx->M == 1 || stride_m == 0 || stride_m >= (long long)ldk * B, "%s: stride_m too small", fn);
  if (B == 0) return AMX_OK;
  hipStream_t s = (hipStream_t)stream;
  if (in_dtype == AMX_IN_F64) {
    hipLaunchKernelGGL(k_assemble<double>, lanes_grid(B), dim3(256), 0, s, (const double*)ob, (const double*)act,
                       ctx->d_norm, act_buf, stride_m, ldk, ctx->S, ctx->A, ctx->M, ctx->k0_pad, B, row_exp,
                       stride_rexp, slot_stride, n_slots);
  } else if (in_dtype == AMX_IN_F32) {
    hipLaunchKernelGGL(k_assemble<float>, lanes_grid(B), dim3(256), 0, s, (const float*)ob, (const float*)act,
                       ctx->d_norm, act_buf, stride_m, ldk, ctx->S, ctx->A, ctx->M, ctx->k0_pad, B, row_exp,
                       stride_rexp, slot_stride, n_slots);
  } else {
    AMX_CHECK_ARG(false, "%s: in_dtype=%d", fn, in_dtype);
  }
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_assemble_input(amx_ctx* ctx, const void* ob, const void* act, int in_dtype, float* act_buf,
                                  long long stride_m, int ldk, int B, void* stream) {
  return assemble("amx_assemble_input", ctx, ob, act, in_dtype, act_buf, stride_m, ldk, B, nullptr, 0, 0, 0,
                  stream);
}

extern "C" int amx_assemble_input_rexp(amx_ctx* ctx, const void* ob, const void* act, int in_dtype, float* act_buf,
                                       long long stride_m, int ldk, int B, int* row_exp, long long strideRexp,
                                       long long slot_stride, int n_slots, void* stream) {
  AMX_CHECK_ARG(row_exp && n_slots >= 1 && n_slots <= 64 &&
                    (slot_stride >= B ? (ctx == nullptr || ctx->M == 1 || strideRexp >= (long long)n_slots * slot_stride)
                                      : blocked_rexp_ok(ctx, B, stride_m, strideRexp, slot_stride, n_slots)),
                "amx_assemble_input_rexp: row_exp=%p n_slots=%d slot_stride=%lld strideRexp=%lld B=%d", (void*)row_exp,
                n_slots, slot_stride, strideRexp, B);
  return assemble("amx_assemble_input_rexp", ctx, ob, act, in_dtype, act_buf, stride_m, ldk, B, row_exp, strideRexp,
                  slot_stride, n_slots, stream);
}

// PolicyArgs of amx_policy_act[_dev] / amx_step_reset_act (ob: null for the fused form, whose
// input rows come from the step kernel), with their argument checks
static int make_policy_args(const char* fn, amx_ctx* ctx, const double* ob, int B, const float* blob, int H1, int H2,
                            const double* noise_scale, const double* noise, uint64_t seed, uint64_t counter,
                            const uint64_t* counter_dev, int eval_mode, double* act, float* mean, float* x0_buf,
                            long long stride_m, int ldk, int* row_exp, long long stride_rexp, long long slot_stride,
                            int n_slots, PolicyArgs& p) {
  AMX_CHECK_ARG(ctx && blob && act, "%s: null pointer", fn);
  AMX_CHECK_ARG(amx::aligned16(blob), "%s: blob must be 16-byte aligned", fn);
  AMX_CHECK_ARG(eval_mode || noise_scale, "%s: noise_scale required unless eval_mode", fn);
  AMX_CHECK_ARG(H1 > 0 && H1 <= POL_MAXH && H2 > 0 && H2 <= POL_MAXH && ctx->A <= POL_MAXH && ctx->S <= POL_MAXH,
                "%s: S=%d H1=%d H2=%d A=%d (max %d)", fn, ctx->S, H1, H2, ctx->A, POL_MAXH);
  AMX_CHECK_ARG(B >= 0, "%s: B=%d", fn, B);
  AMX_CHECK_ARG(!x0_buf || ctx->k0_pad <= POL_X0_COLS, "%s: fused assembly needs k0_pad <= %d (%d)", fn,
                POL_X0_COLS, ctx->k0_pad);
  AMX_CHECK_ARG(!x0_buf || (ctx->have_norm && ldk >= ctx->k0_pad &&
                            (ctx->M == 1 || stride_m == 0 || stride_m >= (long long)ldk * B)),
                "%s: fused assembly needs normalizers and ldk >= k0_pad, stride_m >= ldk*B", fn);
  AMX_CHECK_ARG(!row_exp || (x0_buf && n_slots >= 1 && n_slots <= 64 &&
                             (slot_stride >= B ? (ctx->M == 1 || stride_rexp >= (long long)n_slots * slot_stride)
                                               : blocked_rexp_ok(ctx, B, stride_m, stride_rexp, slot_stride, n_slots))),
                "%s: row_exp needs x0_buf, 1 <= n_slots <= 64, slot_stride >= B (or the member-blocked layout), "
                "stride_rexp", fn);
  const size_t lds = pol_lds_bytes(ctx->S, H1, H2, ctx->A);
  AMX_CHECK_ARG(lds <= 160 * 1024, "%s: S/H too large for LDS staging (%zu B)", fn, lds);
  p.ob = ob; p.blob = blob; p.H1 = H1; p.H2 = H2;
  p.nscale = noise_scale; p.noise = noise;
  p.k0 = (uint32_t)seed; p.k1 = (uint32_t)(seed >> 32); p.ctr_lo = (uint32_t)counter;
  p.ctr_hi = (uint32_t)(counter >> 32); p.eval_mode = eval_mode; p.ctr_dev = counter_dev;
  p.act = act; p.mean_out = mean;
  p.x0 = x0_buf; p.stride_m = stride_m; p.ldk = ldk; p.k0_pad = ctx->k0_pad; p.M = ctx->M; p.norm = ctx->d_norm;
  p.row_exp = row_exp; p.stride_rexp = stride_rexp; p.slot_stride = slot_stride; p.n_slots = n_slots;
  p.S = ctx->S; p.A = ctx->A; p.B = B;
  return AMX_OK;
}

static int policy_act(amx_ctx* ctx, const double* ob, int B, const float* blob, int H1, int H2,
                      const double* noise_scale, const double* noise, uint64_t seed, uint64_t counter,
                      const uint64_t* counter_dev, int eval_mode, double* act, float* mean, float* x0_buf,
                      long long stride_m, int ldk, int* row_exp, long long stride_rexp, long long slot_stride,
                      int n_slots, void* stream) {
  AMX_CHECK_ARG(ob, "amx_policy_act: null ob");
  PolicyArgs p;
  const int rc = make_policy_args("amx_policy_act", ctx, ob, B, blob, H1, H2, noise_scale, noise, seed, counter,
                                  counter_dev, eval_mode, act, mean, x0_buf, stride_m, ldk, row_exp, stride_rexp,
                                  slot_stride, n_slots, p);
  if (rc) return rc;
  if (B == 0) return AMX_OK;
  hipLaunchKernelGGL(k_policy, dim3((B + POL_LANES - 1) / POL_LANES), dim3(256), pol_lds_bytes(ctx->S, H1, H2, ctx->A),
                     (hipStream_t)stream, p);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

struct ResetArgs {  // amx_step_reset's reset half (amx_reset_lanes' arguments)
  const double* table; int R; const int32_t* rows; uint64_t seed; double* ob_out; int32_t* model_idx;
  int32_t* reset_count; int32_t* row_out; int32_t* steps0_out;
  uint64_t* counter; long long counter_delta; double* ob_rec;
};

static int step_impl(amx_ctx* ctx, const float* preds, int ldp, long long strideP, const int32_t* model_idx,
                     const double* ob, double* ob_next, int32_t* num_steps, uint8_t* done, float* disc,
                     float* cost_in, int ldc, int* cost_rexp, uint8_t* nonfinite, int B, void* stream,
                     const ResetArgs* rs = nullptr, const PolicyArgs* pa = nullptr) {
  AMX_CHECK_ARG(ctx && ctx->have_term, "amx_step: context has no termination config");
  AMX_CHECK_ARG(preds && model_idx && ob && ob_next && num_steps && done, "amx_step: null pointer");
  AMX_CHECK_ARG(ldp >= ctx->S && B >= 0, "amx_step: ldp=%d B=%d", ldp, B);
  AMX_CHECK_ARG(!disc || ctx->M >= 2, "amx_step: disagreement needs >= 2 models");
  AMX_CHECK_ARG(!cost_in || ldc >= 2 * ctx->S, "amx_step: ldc=%d < 2S", ldc);
  AMX_CHECK_ARG(ob != ob_next, "amx_step: ob and ob_next must not alias");
  if (B == 0) return AMX_OK;
  StepArgs a;
  a.preds = preds; a.strideP = strideP; a.ldp = ldp;
  a.model_idx = model_idx; a.ob = ob; a.ob_next = ob_next;
  a.num_steps = num_steps; a.done = done; a.disc = disc;
  a.cost_in = cost_in; a.ldc = ldc; a.cost_rexp = cost_rexp; a.nonfinite = nonfinite;
  a.S = ctx->S; a.M = ctx->M; a.B = B; a.term = ctx->term;
  a.model_idx_out = nullptr; a.ob_out = nullptr; a.table = nullptr; a.R = 0; a.rows = nullptr; a.k0 = a.k1 = 0;
  a.reset_count = nullptr; a.row_out = nullptr; a.steps0_out = nullptr; a.counter = nullptr; a.counter_delta = 0;
  a.ob_rec = nullptr;
  if (rs) {
    AMX_CHECK_ARG(rs->table && rs->ob_out && rs->model_idx && rs->reset_count && rs->R > 0,
                  "amx_step_reset: null reset pointer or R=%d", rs->R);
    AMX_CHECK_ARG(rs->ob_out != ob_next && (const int32_t*)rs->model_idx == model_idx,
                  "amx_step_reset: ob_out must differ from ob_next and model_idx be the step's");
    AMX_CHECK_ARG(rs->ob_rec == nullptr || (rs->ob_rec != ob && rs->ob_rec != ob_next && rs->ob_rec != rs->ob_out),
                  "amx_step_reset: ob_rec must be a fourth buffer");
    a.model_idx_out = rs->model_idx; a.ob_out = rs->ob_out; a.table = rs->table; a.R = rs->R; a.rows = rs->rows;
    a.k0 = (uint32_t)rs->seed; a.k1 = (uint32_t)(rs->seed >> 32);
    a.reset_count = rs->reset_count; a.row_out = rs->row_out; a.steps0_out = rs->steps0_out;
    a.counter = rs->counter; a.counter_delta = rs->counter_delta; a.ob_rec = rs->ob_rec;
  }
  const int nit = (ctx->S + 63) / 64;
  if (pa) {  // k_step_act: step t + the policy (and x0 assembly) of step t + 1 on obs[t+1]
    AMX_CHECK_ARG(rs && !rs->counter && !pa->noise && pa->B == B && nit <= 4,
                  "amx_step_reset_act: needs the table reset, no counter advance, no injected noise, S <= 256");
    const size_t lds = pol_lds_bytes(ctx->S, pa->H1, pa->H2, ctx->A) +
                       (size_t)(pol_image_lds_floats(ctx->S, pa->H1, pa->H2, ctx->A) -
                                pol_blob_floats(ctx->S, pa->H1, pa->H2, ctx->A)) * sizeof(float);
    AMX_CHECK_ARG(lds <= 160 * 1024, "amx_step_reset_act: S/H too large for LDS staging (%zu B)", lds);
    const dim3 grid((B + POL_LANES - 1) / POL_LANES);
    switch (nit) {
#define AMX_STEP_ACT_CASE(N)                                                                                       \
  case N:                                                                                                          \
    if (ctx->M == 4 && ctx->step_act_w8) hipLaunchKernelGGL((k_step_act<N, true, true>), grid, dim3(1024), lds,     \
                                                           (hipStream_t)stream, a, *pa);                          \
    else if (ctx->M == 4) hipLaunchKernelGGL((k_step_act<N, true, false>), grid, dim3(1024), lds, (hipStream_t)stream, \
                                             a, *pa);                                                              \
    else hipLaunchKernelGGL((k_step_act<N, false, false>), grid, dim3(1024), lds, (hipStream_t)stream, a, *pa);   \
    break;
      AMX_STEP_ACT_CASE(1) AMX_STEP_ACT_CASE(2) AMX_STEP_ACT_CASE(3) AMX_STEP_ACT_CASE(4)
#undef AMX_STEP_ACT_CASE
    }
    AMX_CHECK_LAUNCH();
    return AMX_OK;
  }
  switch (nit) {
#define AMX_STEP_CASE(N)                                                                                 \
  case N:                                                                                                \
    if (ctx->M == 4) hipLaunchKernelGGL((k_step<N, true>), lanes_grid(B), dim3(256), 0, (hipStream_t)stream, a); \
    else hipLaunchKernelGGL((k_step<N, false>), lanes_grid(B), dim3(256), 0, (hipStream_t)stream, a);     \
    break;
    AMX_STEP_CASE(1) AMX_STEP_CASE(2) AMX_STEP_CASE(3) AMX_STEP_CASE(4)
    AMX_STEP_CASE(5) AMX_STEP_CASE(6) AMX_STEP_CASE(7) AMX_STEP_CASE(8)
#undef AMX_STEP_CASE
    default: AMX_CHECK_ARG(false, "amx_step: S=%d exceeds 512", ctx->S);
  }
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_step(amx_ctx* ctx, const float* preds, int ldp, long long strideP, const int32_t* model_idx,
                        const double* ob, double* ob_next, int32_t* num_steps, uint8_t* done, float* disc,
                        float* cost_in, int ldc, uint8_t* nonfinite, int B, void* stream) {
  return step_impl(ctx, preds, ldp, strideP, model_idx, ob, ob_next, num_steps, done, disc, cost_in, ldc, nullptr,
                   nonfinite, B, stream);
}

extern "C" int amx_step_rexp(amx_ctx* ctx, const float* preds, int ldp, long long strideP, const int32_t* model_idx,
                             const double* ob, double* ob_next, int32_t* num_steps, uint8_t* done, float* disc,
                             float* cost_in, int ldc, int* cost_rexp, uint8_t* nonfinite, int B, void* stream) {
  AMX_CHECK_ARG(cost_in && cost_rexp, "amx_step_rexp: cost_in and cost_rexp are required");
  return step_impl(ctx, preds, ldp, strideP, model_idx, ob, ob_next, num_steps, done, disc, cost_in, ldc, cost_rexp,
                   nonfinite, B, stream);
}

extern "C" int amx_step_reset(amx_ctx* ctx, const float* preds, int ldp, long long strideP, int32_t* model_idx,
                              const double* ob, double* ob_next, int32_t* num_steps, uint8_t* done, float* disc,
                              float* cost_in, int ldc, int* cost_rexp, uint8_t* nonfinite, const double* table,
                              int R, const int32_t* rows, uint64_t seed, double* ob_out, int32_t* reset_count,
                              int32_t* row_out, int32_t* steps0_out, uint64_t* counter, long long counter_delta,
                              double* ob_rec, int B, void* stream) {
  AMX_CHECK_ARG(!cost_rexp || cost_in, "amx_step_reset: cost_rexp needs cost_in");
  const ResetArgs rs = {table, R, rows, seed, ob_out, model_idx, reset_count, row_out, steps0_out, counter,
                        counter_delta, ob_rec};
  return step_impl(ctx, preds, ldp, strideP, model_idx, ob, ob_next, num_steps, done, disc, cost_in, ldc, cost_rexp,
                   nonfinite, B, stream, &rs);
}

extern "C" int amx_step_reset_act(amx_ctx* ctx, const float* preds, int ldp, long long strideP, int32_t* model_idx,
                                  const double* ob, double* ob_next, int32_t* num_steps, uint8_t* done, float* disc,
                                  float* cost_in, int ldc, int* cost_rexp, uint8_t* nonfinite, const double* table,
                                  int R, const int32_t* rows, uint64_t seed, double* ob_out, int32_t* reset_count,
                                  int32_t* row_out, int32_t* steps0_out, double* ob_rec, const float* blob, int H1,
                                  int H2, const double* noise_scale, uint64_t policy_seed, uint64_t counter,
                                  const uint64_t* counter_dev, int eval_mode, double* act, float* mean,
                                  float* x0_buf, long long stride_m, int ldk, int* row_exp, long long stride_rexp,
                                  long long slot_stride, int n_slots, int B, void* stream) {
  AMX_CHECK_ARG(!cost_rexp || cost_in, "amx_step_reset_act: cost_rexp needs cost_in");
  PolicyArgs p;
  int rc = make_policy_args("amx_step_reset_act", ctx, nullptr, B, blob, H1, H2, noise_scale, nullptr, policy_seed,
                            counter, counter_dev, eval_mode, act, mean, x0_buf, stride_m, ldk, row_exp, stride_rexp,
                            slot_stride, n_slots, p);
  if (rc) return rc;
  const ResetArgs rs = {table, R, rows, seed, ob_out, model_idx, reset_count, row_out, steps0_out, nullptr, 0,
                        ob_rec};
  return step_impl(ctx, preds, ldp, strideP, model_idx, ob, ob_next, num_steps, done, disc, cost_in, ldc, cost_rexp,
                   nonfinite, B, stream, &rs, &p);
}

extern "C" int amx_disagreement(amx_ctx* ctx, const float* preds, int ldp, long long strideP, float* disc, int B,
                                void* stream) {
  AMX_CHECK_ARG(ctx && preds && disc, "amx_disagreement: null pointer");
  AMX_CHECK_ARG(ctx->M >= 2, "amx_disagreement: needs >= 2 models (M=%d)", ctx->M);
  AMX_CHECK_ARG(ldp >= ctx->S && B >= 0, "amx_disagreement: ldp=%d B=%d", ldp, B);
  if (B == 0) return AMX_OK;
  hipLaunchKernelGGL(k_disagreement, lanes_grid(B), dim3(256), 0, (hipStream_t)stream, preds, strideP, ldp, disc,
                     ctx->S, ctx->M, B);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_reset_lanes(amx_ctx* ctx, const uint8_t* mask, const double* table, int R, const int32_t* rows,
                               uint64_t seed, const double* ob_src, double* ob_out, int32_t* num_steps,
                               int32_t* model_idx, int32_t* reset_count, int32_t* row_out, int B, void* stream) {
  AMX_CHECK_ARG(ctx && table && ob_out && num_steps && model_idx && reset_count, "amx_reset_lanes: null pointer");
  AMX_CHECK_ARG(R > 0 && B >= 0, "amx_reset_lanes: R=%d B=%d", R, B);
  AMX_CHECK_ARG(mask == nullptr || ob_src != nullptr, "amx_reset_lanes: masked reset needs ob_src");
  if (B == 0) return AMX_OK;
  hipLaunchKernelGGL(k_reset, lanes_grid(B), dim3(256), 0, (hipStream_t)stream, mask, table, R, rows,
                     (uint32_t)seed, (uint32_t)(seed >> 32), ob_src, ob_out, num_steps, model_idx, reset_count,
                     row_out, ctx->S, ctx->M, B);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" long long amx_policy_blob_floats(const amx_ctx* ctx, int H1, int H2) {
  if (!ctx || H1 <= 0 || H2 <= 0) return -1;
  return pol_image_lds_floats(ctx->S, H1, H2, ctx->A);  // whole 1-KiB pieces (k_step_act's LDS-DMA)
}

extern "C" int amx_policy_pack(amx_ctx* ctx, const float* W1, const float* b1, int H1, const float* W2,
                               const float* b2, int H2, const float* W3, const float* b3, float* blob,
                               void* stream) {
  AMX_CHECK_ARG(ctx && W1 && b1 && W2 && b2 && W3 && b3 && blob, "amx_policy_pack: null pointer");
  AMX_CHECK_ARG(H1 > 0 && H1 <= POL_MAXH && H2 > 0 && H2 <= POL_MAXH && ctx->A <= POL_MAXH,
                "amx_policy_pack: H1=%d H2=%d A=%d (max %d)", H1, H2, ctx->A, POL_MAXH);
  AMX_CHECK_ARG(amx::aligned16(blob), "amx_policy_pack: blob must be 16-byte aligned");
  const int n = pol_blob_floats(ctx->S, H1, H2, ctx->A);
  hipLaunchKernelGGL(k_policy_pack, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, W1, b1, H1, W2, b2,
                     H2, W3, b3, ctx->S, ctx->A, blob);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_policy_act(amx_ctx* ctx, const double* ob, int B, const float* blob, int H1, int H2,
                              const double* noise_scale, const double* noise, uint64_t seed, uint64_t counter,
                              int eval_mode, double* act, float* mean, float* x0_buf, long long stride_m, int ldk,
                              int* row_exp, long long stride_rexp, long long slot_stride, int n_slots,
                              void* stream) {
  return policy_act(ctx, ob, B, blob, H1, H2, noise_scale, noise, seed, counter, nullptr, eval_mode, act, mean,
                    x0_buf, stride_m, ldk, row_exp, stride_rexp, slot_stride, n_slots, stream);
}

extern "C" int amx_policy_act_dev(amx_ctx* ctx, const double* ob, int B, const float* blob, int H1, int H2,
                                  const double* noise_scale, const double* noise, uint64_t seed,
                                  const uint64_t* counter, uint64_t counter_offset, int eval_mode, double* act,
                                  float* mean, float* x0_buf, long long stride_m, int ldk, int* row_exp,
                                  long long stride_rexp, long long slot_stride, int n_slots, void* stream) {
  AMX_CHECK_ARG(counter, "amx_policy_act_dev: null counter");
  return policy_act(ctx, ob, B, blob, H1, H2, noise_scale, noise, seed, counter_offset, counter, eval_mode, act,
                    mean, x0_buf, stride_m, ldk, row_exp, stride_rexp, slot_stride, n_slots, stream);
}

__global__ void k_counter_add(uint64_t* c, long long d) { c[0] += (uint64_t)d; }

// *counter += delta when the stream reaches this launch (a captured rollout's policy counter)
extern "C" int amx_counter_add(amx_ctx* ctx, uint64_t* counter, long long delta, void* stream) {
  AMX_CHECK_ARG(ctx && counter, "amx_counter_add: null pointer");
  hipLaunchKernelGGL(k_counter_add, dim3(1), dim3(1), 0, (hipStream_t)stream, counter, delta);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_philox(amx_ctx* ctx, uint64_t seed, uint32_t ctr1, uint32_t ctr2, uint32_t ctr3, uint32_t* out,
                          int n, void* stream) {
  AMX_CHECK_ARG(ctx && out && n >= 0, "amx_philox: bad argument");
  if (n == 0) return AMX_OK;
  hipLaunchKernelGGL(k_philox, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, (uint32_t)seed,
                     (uint32_t)(seed >> 32), ctr1, ctr2, ctr3, out, n);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_set_step_act_occupancy(amx_ctx* ctx, int two_per_cu) {
  AMX_CHECK_ARG(ctx, "amx_set_step_act_occupancy: null ctx");
  ctx->step_act_w8 = two_per_cu ? 1 : 0;
  return AMX_OK;
}
