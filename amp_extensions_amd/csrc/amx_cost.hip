// Reward kernels of the relabel block (mjrl/mjrl/algos/batch_reinforce.py:103-169):
// ordered fp64 reduction of the RFF feature-sum partials, the closed-form MMD witness
// (RBFLinearCost.fit_cost), the per-sample pessimistic MMD reward (get_costs +
// get_bonus_costs), the expert cost, and the AMP least-squares discriminator reward.
//
// All are HBM-bound streaming passes over per-sample rows (phi rows are 2 KB); one wave
// per row, float4 loads, fp64 wave reductions.  Built with -ffp-contract=off so the
// scalar reward algebra rounds exactly like the reference's separate torch fp32 ops.
#include "amx_common.h"

namespace {

// fp64 DPP move of both halves (lanes outside row_mask keep 0.0)
template <int CTRL, int RM>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, RM, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, RM, 0xf, false);
  return __hiloint2double(hi, lo);
}

// Sum over the wave's 64 lanes, returned to every lane, on the DPP path (no LDS traffic; the
// same fixed association as amx_step.hip's): quad xor 1, 2, the 8- and 16-lane mirrors, rows
// 0 -> 1, 2 -> 3 (row_bcast:15), rows 0+1 -> 2, 3 (row_bcast:31), lane 63 read back.
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

// out[f] = sum_p partials[p][f].  Block = 64 columns x 16 waves; wave w sums its contiguous
// chunk of parts in ascending order, then the 16 chunk sums are added in wave order:
// the result is deterministic (fixed association) and the dependent-add chain is n/16 long.
// Column sums of fp64 partial rows [n_parts][F] in a fixed order: a 1024-thread block per 16
// columns, thread (g = t / 16, c = t % 16) summing the contiguous run of rows g*per .. of column
// c in row order (64 runs per column: 20 rows each for the 40 960-row rollout's 1280 partial
// rows, where 16 runs of 80 rows made the pass a chain of ten load round trips on 8 CUs), then
// the 64 run sums added in run order.  Shared by k_sum_partials and k_feature_message, so both
// give the same bits.
constexpr int CS_COLS = 16, CS_RUNS = 64;
__device__ inline void colsum_parts(const double* __restrict__ partials, int n_parts, int F, double* __restrict__ out) {
  __shared__ double red[CS_RUNS][CS_COLS];
  const int c = threadIdx.x % CS_COLS, g = threadIdx.x / CS_COLS;
  const int f = blockIdx.x * CS_COLS + c;
  const int per = (n_parts + CS_RUNS - 1) / CS_RUNS;
  const int p0 = g * per, p1 = min(n_parts, p0 + per);
  double s = 0.0;
  if (f < F) {
#pragma unroll 8
    for (int p = p0; p < p1; ++p) s += partials[(long long)p * F + f];  // 8 loads in flight, same add order
  }
  red[g][c] = s;
  __syncthreads();
  if (g == 0 && f < F) {
    double t = 0.0;
#pragma unroll 8
    for (int i = 0; i < CS_RUNS; ++i) t += red[i][c];
    out[f] = t;
  }
}

__global__ __launch_bounds__(1024) void k_sum_partials(const double* __restrict__ partials, int n_parts, int F,
                                                       double* __restrict__ out) {
  colsum_parts(partials, n_parts, F, out);
}

// w = (float)(sum/count) - phi_e ; mmd = dot(w, w).  One block; F <= 4096.
__global__ __launch_bounds__(256) void k_mmd_fit(const double* __restrict__ phi_sum, double count,
                                                 const float* __restrict__ phi_e, int F, float* __restrict__ w,
                                                 float* __restrict__ mmd) {
  __shared__ double red[4];
  double acc = 0.0;
  if (count == 0.0) count = phi_sum[F];  // the fused [sum phi | count] message
  for (int f = threadIdx.x; f < F; f += blockDim.x) {
    const float mean = (float)(phi_sum[f] / count);
    const float wf = mean - phi_e[f];
    w[f] = wf;
    acc += (double)wf * (double)wf;
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) *mmd = (float)(red[0] + red[1] + red[2] + red[3]);
}

// dot(phi[row], w) over F (F % 256 == 0 handled by float4 x 64 lanes per 256 floats)
__device__ inline double row_dot(const float* __restrict__ row, const float* __restrict__ w, int F, int lane) {
  double s = 0.0;
  for (int f = lane * 4; f < F; f += 256) {
    const float4 p = *reinterpret_cast<const float4*>(row + f);
    const float4 q = *reinterpret_cast<const float4*>(w + f);
    s += (double)p.x * q.x + (double)p.y * q.y + (double)p.z * q.z + (double)p.w * q.w;
  }
  return wave_sum(s);
}

__device__ inline float clampf_ref(float v, float lo, float hi) {
  // torch.clamp(min, max): min first, then max; NaN propagates
  if (v != v) return v;
  v = v < lo ? lo : v;
  return v > hi ? hi : v;
}

// CLAMP: cost_range given (clamped cost, bonus = min(disc/thr, 1) * c_min);
// !CLAMP: cost_range None (raw cost, bonus = raw disagreement, linear_cost.py:103, 138-139).
template <bool CLAMP>
__global__ __launch_bounds__(256) void k_mmd_reward(const float* __restrict__ phi, int ldphi,
                                                    const float* __restrict__ w, int F,
                                                    const float* __restrict__ disc, float thr, float one_m_lambda,
                                                    float lambda_b, float c_min, float c_max,
                                                    float* __restrict__ reward, float* __restrict__ ipm_out,
                                                    float* __restrict__ wb_out, int n) {
  const int r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= n) return;
  const double dot = row_dot(phi + (long long)r * ldphi, w, F, lane);
  if (lane != 0) return;
  float v, bonus;
  if constexpr (CLAMP) {
    v = clampf_ref((float)dot, c_min, c_max);                  // linear_cost.py:102
    float dh = disc[r] / thr;                                  // :132
    if (dh > 1.0f) dh = 1.0f;                                  // :134
    bonus = dh * c_min;                                        // :136
  } else {
    v = (float)dot;                                            // :103
    bonus = disc[r];                                           // :139
  }
  const float ipm = one_m_lambda * v;                          // :141  (1-lambda)*rff_cost
  const float wb = lambda_b * bonus;                           // :144
  const float cost = ipm - wb;                                 // :147
  reward[r] = -1.0f * cost;                                    // batch_reinforce.py:144
  if (ipm_out) ipm_out[r] = ipm;
  if (wb_out) wb_out[r] = wb;
}

// Block partial of sum clamp(phi_E[r].w): 4 rows per block-iteration (one per wave),
// grid-stride; partials[block] in fp64, then an ordered sum.
__global__ __launch_bounds__(256) void k_expert_cost(const float* __restrict__ phi, int ldphi,
                                                     const float* __restrict__ w, int F, int n, float c_min,
                                                     float c_max, double* __restrict__ partials) {
  __shared__ double red[4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double acc = 0.0;
  for (int r = blockIdx.x * 4 + wave; r < n; r += gridDim.x * 4) {
    const double dot = row_dot(phi + (long long)r * ldphi, w, F, lane);
    acc += (double)clampf_ref((float)dot, c_min, c_max);
  }
  if (lane == 0) red[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partials[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// Deterministic sum of n partials: thread t sums t, t+256, ... then a fixed-shape tree.
__global__ __launch_bounds__(256) void k_sum_small(const double* __restrict__ partials, int n,
                                                   double* __restrict__ out, float* __restrict__ mean_out = nullptr,
                                                   int n_rows = 1, float scale = 1.f) {
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += partials[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = red[0];
    if (mean_out) mean_out[0] = scale * (float)(red[0] / (double)n_rows);  // fp32 product, as torch
  }
}

// ---- the relabel tail in one launch --------------------------------------------------------
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) uint32_t gu32c;

// Batched row dots for the relabel: NC = F/256 float4 chunks per lane (lane l reads floats
// 4l + 256c of a row, exactly row_dot's per-lane order, then the same wave butterfly), R rows
// loaded per wave before any arithmetic so one memory round trip serves R rows (row_dot waits
// one trip per row).  The per-row result has row_dot's bits; NC = 0 is the generic-F path.
template <int NC>
constexpr int relabel_rows() { return NC == 0 ? 1 : (8 / NC > 0 ? 8 / NC : 1); }

template <int NC, int R>
__device__ inline void rows_load(const float* __restrict__ base, int ld, int r0, int step, int nrows, int lane,
                                 float4 (&p)[R][NC > 0 ? NC : 1]) {
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int r = r0 + i * step;
#pragma unroll
    for (int c = 0; c < (NC > 0 ? NC : 1); ++c)
      p[i][c] = (NC > 0 && r < nrows) ? *reinterpret_cast<const float4*>(base + (long long)r * ld + lane * 4 + 256 * c)
                                      : float4{0.f, 0.f, 0.f, 0.f};
  }
}

template <int NC, int R>
__device__ inline void rows_dot(const float4 (&p)[R][NC > 0 ? NC : 1], const float* __restrict__ base, int ld,
                                int r0, int step, int nrows, const float* __restrict__ w, int F, int lane,
                                double (&d)[R]) {
  if constexpr (NC == 0) {  // generic F: one row at a time (row_dot)
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int r = r0 + i * step;
      d[i] = r < nrows ? row_dot(base + (long long)r * ld, w, F, lane) : 0.0;
    }
  } else {
    float4 q[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) q[c] = *reinterpret_cast<const float4*>(w + lane * 4 + 256 * c);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double s = 0.0;
#pragma unroll
      for (int c = 0; c < NC; ++c)
        s += (double)p[i][c].x * q[c].x + (double)p[i][c].y * q[c].y + (double)p[i][c].z * q[c].z +
             (double)p[i][c].w * q[c].w;
      d[i] = s;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) d[i] = wave_sum(d[i]);  // row_dot's reduction
  }
}

// k_mmd_relabel = k_mmd_fit + k_mmd_reward + k_expert_cost + k_sum_small: every block derives
// the witness w from the (all-reduced) [sum phi | count] message into LDS (the same fp64
// divide and fp32 subtraction as k_mmd_fit, so every block holds identical bits); block 0 also
// publishes w and w.w; blocks [0, ne) take the expert rows b*4 + wave + k*4ne (k_expert_cost's
// assignment and per-wave order, R per round trip), blocks [ne, ne + nr) score R rollout rows
// per wave.  Each wave issues its first rows' loads before the witness prologue.  The
// expert partials are handed to the last-arriving expert block (agent-scope counter,
// cdna_hip_programming.md §5 split-K form: sc1 partial stores drained before the relaxed
// counter add, one acquire in the reducer), which sums them in index order (deterministic)
// and resets the counter for the next launch.
struct RelabelArgs {
  const double* msg; double count; const float* phi_e; int F;
  float* w; float* mmd;
  const float* phi; int ldphi; const float* disc; float thr, one_m_lambda, lambda_b, c_min, c_max;
  float* reward; float* ipm; float* wb; int n, nr;
  const float* erows; int lde, ne_rows, ne;  // expert rows (null: no expert cost)
  double* eout;                               // [0] sum, [1 .. ne] block partials
  float* emean; float escale; uint32_t* counter;
};

template <bool CLAMP, int NC>
__global__ __launch_bounds__(256) void k_mmd_relabel(RelabelArgs a) {
  constexpr int R = relabel_rows<NC>();
  extern __shared__ __attribute__((aligned(16))) float wsh[];  // [F]
  __shared__ double red[256];
  __shared__ int last;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  // blocks [0, ne) take the expert rows (several row batches each: dispatched first, so their
  // longer chains overlap the rollout blocks instead of trailing them), [ne, ne + nr) the
  // rollout rows (one batch each)
  const bool roll = (int)blockIdx.x >= a.ne;
  // this wave's first rows, in flight during the prologue
  const int eb = roll ? 0 : (int)blockIdx.x;
  const int rb = roll ? (int)blockIdx.x - a.ne : 0;
  const int r0 = roll ? (rb * 4 + wave) * R : eb * 4 + wave;
  const int step = roll ? 1 : a.ne * 4;
  const float* base = roll ? a.phi : a.erows;
  const int ld = roll ? a.ldphi : a.lde;
  const int nrows = roll ? a.n : a.ne_rows;
  float4 p[R][NC > 0 ? NC : 1];
  rows_load<NC, R>(base, ld, r0, step, nrows, lane, p);
  double count = a.count == 0.0 ? a.msg[a.F] : a.count;
  double acc = 0.0;
  for (int f = t; f < a.F; f += 256) {
    const float mean = (float)(a.msg[f] / count);
    const float wf = mean - a.phi_e[f];
    wsh[f] = wf;
    acc += (double)wf * (double)wf;
  }
  if (blockIdx.x == 0) {
    for (int f = t; f < a.F; f += 256) a.w[f] = wsh[f];
    acc = wave_sum(acc);
    if (lane == 0) red[wave] = acc;
  }
  __syncthreads();
  if (blockIdx.x == 0 && t == 0) *a.mmd = (float)(red[0] + red[1] + red[2] + red[3]);
  if (roll) {  // rollout rows r0 .. r0 + R - 1
    double d[R];
    rows_dot<NC, R>(p, base, ld, r0, 1, nrows, wsh, a.F, lane, d);
    if (lane != 0) return;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int r = r0 + i;
      if (r >= a.n) break;
      float v, bonus;
      if constexpr (CLAMP) {
        v = clampf_ref((float)d[i], a.c_min, a.c_max);           // linear_cost.py:102
        float dh = a.disc[r] / a.thr;                            // :132
        if (dh > 1.0f) dh = 1.0f;                                // :134
        bonus = dh * a.c_min;                                    // :136
      } else {
        v = (float)d[i];                                         // :103
        bonus = a.disc[r];                                       // :139
      }
      const float ipm = a.one_m_lambda * v;                      // :141
      const float wbv = a.lambda_b * bonus;                      // :144
      const float cost = ipm - wbv;                              // :147
      a.reward[r] = -1.0f * cost;                                // batch_reinforce.py:144
      if (a.ipm) a.ipm[r] = ipm;
      if (a.wb) a.wb[r] = wbv;
    }
    return;
  }
  if (a.ne == 0) return;
  // expert rows: sum clamp(phi_E[r].w) (linear_cost.py:105-109), rows in k_expert_cost's order;
  // two row batches in flight (the next batch's loads are issued before the current one's dots)
  double e = 0.0;
  float4 p2[R][NC > 0 ? NC : 1];
  auto consume = [&](const float4 (&pp)[R][NC > 0 ? NC : 1], int rb) {
    double d[R];
    rows_dot<NC, R>(pp, base, ld, rb, step, nrows, wsh, a.F, lane, d);
#pragma unroll
    for (int i = 0; i < R; ++i)
      if (rb + i * step < a.ne_rows) e += (double)clampf_ref((float)d[i], a.c_min, a.c_max);
  };
  for (int rb = r0; rb < a.ne_rows;) {
    const int rn = rb + R * step;
    if (rn < a.ne_rows) rows_load<NC, R>(base, ld, rn, step, nrows, lane, p2);
    consume(p, rb);
    if (rn >= a.ne_rows) break;
    rb = rn + R * step;
    if (rb < a.ne_rows) rows_load<NC, R>(base, ld, rb, step, nrows, lane, p);
    consume(p2, rn);
  }
  __syncthreads();  // red[] reuse
  if (lane == 0) red[wave] = e;
  __syncthreads();
  if (t == 0) {
    const double part = red[0] + red[1] + red[2] + red[3];
    __hip_atomic_store((gu64*)(a.eout + 1 + eb), __double_as_longlong(part), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add((gu32c*)a.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           (uint32_t)(a.ne - 1);
    if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  if (!last) return;
  double s = 0.0;  // ordered: thread t sums t, t + 256, ...; then the fixed tree of k_sum_small
  for (int i = t; i < a.ne; i += 256)
    s += __longlong_as_double(__hip_atomic_load((const gu64*)(a.eout + 1 + i), __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT));
  red[t] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  if (t == 0) {
    a.eout[0] = red[0];
    if (a.emean) a.emean[0] = a.escale * (float)(red[0] / (double)a.ne_rows);  // fp32 product, as torch
    __hip_atomic_store((gu32c*)a.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// [sum phi | count]: the fp64 column sums of the RFF partials (as k_sum_partials) and the
// sample count in slot F of the same message, so the all-reduce / fit read one buffer.
__global__ __launch_bounds__(1024) void k_feature_message(const double* __restrict__ partials, int n_parts, int F,
                                                          double count, double* __restrict__ out) {
  colsum_parts(partials, n_parts, F, out);
  if (blockIdx.x == 0 && threadIdx.x == 0) out[F] = count;
}

// LOSS 0: least squares (get_ls_costs, gail_cost.py:231-236); LOSS 1: log-likelihood
// (get_ll_costs, :238-244: cost = logsigmoid(D)).
template <int LOSS>
__global__ __launch_bounds__(256) void k_amp_reward(const float* __restrict__ h, int ldh, int Hd,
                                                    const float* __restrict__ w3, float b3,
                                                    const float* __restrict__ disc, float one_m_lambda,
                                                    float lambda_b, float* __restrict__ reward,
                                                    float* __restrict__ logits, int n) {
  const int r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= n) return;
  double s = 0.0;
  const float* row = h + (long long)r * ldh;
  for (int k = lane; k < Hd; k += 64) s += (double)row[k] * (double)w3[k];
  s = wave_sum(s);
  if (lane != 0) return;
  const float D = (float)s + b3;                     // Discriminator last nn.Linear
  float rew;
  if constexpr (LOSS == 0) {
    const float om = 1.0f - D;                       // gail_cost.py:234  1.0 - disc_outs
    const float sq = om * om;                        //                   (.)**2
    const float q = 0.25f * sq;                      //                   0.25 * (.)
    rew = 1.0f - q;                                  //                   1.0 - (.)
    if (rew < 0.0f) rew = 0.0f;                      // :235
  } else {
    // F.logsigmoid = min(D, 0) - log1p(exp(-|D|)); reward = -cost
    rew = -(fminf(D, 0.0f) - log1pf(expf(-fabsf(D))));
  }
  if (logits) logits[r] = D;
  if (disc == nullptr) {                             // get_costs path: reward = -cost = r
    reward[r] = rew;
    return;
  }
  const float input_cost = -rew;                     // :236 (ll: logsigmoid(D), :243)
  const float ipm = one_m_lambda * input_cost;       // :269
  const float bonus = lambda_b * disc[r];            // :273 (raw disagreement)
  const float cost = ipm - bonus;                    // :275
  reward[r] = -1.0f * cost;                          // batch_reinforce.py:144
}

}  // namespace

extern "C" int amx_sum_partials(amx_ctx* ctx, const double* partials, int n_parts, int F, double* out,
                                void* stream) {
  AMX_CHECK_ARG(ctx && partials && out && n_parts >= 0 && F > 0, "amx_sum_partials: bad argument");
  hipLaunchKernelGGL(k_sum_partials, dim3((F + CS_COLS - 1) / CS_COLS), dim3(1024), 0, (hipStream_t)stream, partials,
                     n_parts, F, out);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_mmd_fit(amx_ctx* ctx, const double* phi_sum, double count, const float* phi_e, int F,
                           float* w, float* mmd, void* stream) {
  AMX_CHECK_ARG(ctx && phi_sum && phi_e && w && mmd && F > 0, "amx_mmd_fit: bad argument");
  AMX_CHECK_ARG(count > 0.0 || count == 0.0, "amx_mmd_fit: count must be positive (empty rollout), or 0: read phi_sum[F]");
  hipLaunchKernelGGL(k_mmd_fit, dim3(1), dim3(256), 0, (hipStream_t)stream, phi_sum, count, phi_e, F, w, mmd);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

static int mmd_reward(bool clamp, amx_ctx* ctx, const float* phi, int ldphi, const float* w, int F, const float* disc,
                      float thr, double lambda_b, float c_min, float c_max, float* reward, float* ipm, float* wbonus,
                      int n, void* stream) {
  AMX_CHECK_ARG(ctx && phi && w && disc && reward, "amx_mmd_reward: null pointer");
  AMX_CHECK_ARG(F > 0 && F % 256 == 0 && ldphi >= F && ldphi % 4 == 0, "amx_mmd_reward: F=%d ldphi=%d", F, ldphi);
  AMX_CHECK_ARG(amx::aligned16(phi) && amx::aligned16(w), "amx_mmd_reward: phi/w must be 16-byte aligned");
  AMX_CHECK_ARG(n >= 0, "amx_mmd_reward: n=%d", n);
  if (n == 0) return AMX_OK;
  // lambda is a Python double in the reference: (1 - lambda) is formed in double, then
  // torch rounds each scalar to float32 for the fp32 kernel (linear_cost.py:141,144).
  const float one_m_lambda = (float)(1.0 - lambda_b);
  if (clamp)
    hipLaunchKernelGGL(k_mmd_reward<true>, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, phi, ldphi, w, F,
                       disc, thr, one_m_lambda, (float)lambda_b, c_min, c_max, reward, ipm, wbonus, n);
  else
    hipLaunchKernelGGL(k_mmd_reward<false>, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, phi, ldphi, w, F,
                       disc, thr, one_m_lambda, (float)lambda_b, c_min, c_max, reward, ipm, wbonus, n);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_mmd_reward(amx_ctx* ctx, const float* phi, int ldphi, const float* w, int F, const float* disc,
                              float thr, double lambda_b, float c_min, float c_max, float* reward, float* ipm,
                              float* wbonus, int n, void* stream) {
  return mmd_reward(true, ctx, phi, ldphi, w, F, disc, thr, lambda_b, c_min, c_max, reward, ipm, wbonus, n, stream);
}

extern "C" int amx_mmd_reward_raw(amx_ctx* ctx, const float* phi, int ldphi, const float* w, int F, const float* disc,
                                  double lambda_b, float* reward, float* ipm, float* wbonus, int n, void* stream) {
  return mmd_reward(false, ctx, phi, ldphi, w, F, disc, 1.0f, lambda_b, 0.f, 0.f, reward, ipm, wbonus, n, stream);
}

// Blocks of the expert-cost reduction over n rows (k_expert_cost and k_mmd_relabel share it, so
// both sum the same block partials in the same order): 16 rows per block (4 waves x one batch),
// at most 1024 blocks (grid-stride beyond: 50 000 rows -> 1024 blocks; a rank's 6 250-row shard
// -> 391 instead of 1024 blocks of mostly idle waves).
static int expert_blocks(int n) {
  const int b = (n + 15) / 16;
  return b < 1024 ? (b > 0 ? b : 1) : 1024;
}

extern "C" int amx_expert_cost(amx_ctx* ctx, const float* phi_e_rows, int ldphi, const float* w, int F, int n,
                               float c_min, float c_max, double* out, float* mean_out, double lambda_b,
                               void* stream) {
  AMX_CHECK_ARG(ctx && phi_e_rows && w && out, "amx_expert_cost: null pointer");
  AMX_CHECK_ARG(F > 0 && F % 256 == 0 && ldphi >= F && ldphi % 4 == 0, "amx_expert_cost: F=%d ldphi=%d", F, ldphi);
  AMX_CHECK_ARG(n > 0, "amx_expert_cost: n=%d", n);
  // partials live in out[1 .. nb]; out must hold 1 + 1024 doubles
  const int nb = expert_blocks(n);
  hipLaunchKernelGGL(k_expert_cost, dim3(nb), dim3(256), 0, (hipStream_t)stream, phi_e_rows, ldphi, w, F, n, c_min,
                     c_max, out + 1);
  AMX_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_sum_small, dim3(1), dim3(256), 0, (hipStream_t)stream, out + 1, nb, out, mean_out, n,
                     (float)(1.0 - lambda_b));
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_disc_reward(amx_ctx* ctx, int loss_type, const float* h, int ldh, int Hd, const float* w3,
                               float b3, const float* disc, double lambda_b, float* reward, float* logits, int n,
                               void* stream) {
  AMX_CHECK_ARG(ctx && h && w3 && reward, "amx_disc_reward: null pointer");
  AMX_CHECK_ARG(Hd > 0 && ldh >= Hd && n >= 0, "amx_disc_reward: Hd=%d ldh=%d n=%d", Hd, ldh, n);
  AMX_CHECK_ARG(loss_type == AMX_DISC_LEAST_SQUARES || loss_type == AMX_DISC_LOG_LIKELIHOOD,
                "amx_disc_reward: loss_type=%d", loss_type);
  if (n == 0) return AMX_OK;
  const float one_m_lambda = (float)(1.0 - lambda_b);
  if (loss_type == AMX_DISC_LEAST_SQUARES)
    hipLaunchKernelGGL(k_amp_reward<0>, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, h, ldh, Hd, w3, b3,
                       disc, one_m_lambda, (float)lambda_b, reward, logits, n);
  else
    hipLaunchKernelGGL(k_amp_reward<1>, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, h, ldh, Hd, w3, b3,
                       disc, one_m_lambda, (float)lambda_b, reward, logits, n);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_amp_reward(amx_ctx* ctx, const float* h, int ldh, int Hd, const float* w3, float b3,
                              const float* disc, double lambda_b, float* reward, float* logits, int n,
                              void* stream) {
  return amx_disc_reward(ctx, AMX_DISC_LEAST_SQUARES, h, ldh, Hd, w3, b3, disc, lambda_b, reward, logits, n, stream);
}

// out[b] = float32 [x0[b, :w0], x1[b, :w1], x2[b, :w2], 0 ...] up to ldc: the cost-input row
// of every input type (linear_cost.py:115-127, gail_cost.py:258-268).  One wave per row.
__global__ __launch_bounds__(256) void k_cost_rows(const double* __restrict__ x0, long long ld0, int w0,
                                                   const double* __restrict__ x1, long long ld1, int w1,
                                                   const double* __restrict__ x2, long long ld2, int w2, int B,
                                                   float* __restrict__ out, int ldc) {
  const int r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= B) return;
  float* o = out + (long long)r * ldc;
  for (int j = lane; j < ldc; j += 64) {
    float v = 0.f;
    if (j < w0) v = (float)x0[(long long)r * ld0 + j];
    else if (j < w0 + w1) v = (float)x1[(long long)r * ld1 + (j - w0)];
    else if (j < w0 + w1 + w2) v = (float)x2[(long long)r * ld2 + (j - w0 - w1)];
    o[j] = v;
  }
}

extern "C" int amx_cost_rows(amx_ctx* ctx, const double* x0, long long ld0, int w0, const double* x1, long long ld1,
                             int w1, const double* x2, long long ld2, int w2, int B, float* out, int ldc,
                             void* stream) {
  AMX_CHECK_ARG(ctx && out && B >= 0, "amx_cost_rows: bad arguments");
  AMX_CHECK_ARG(w0 >= 0 && w1 >= 0 && w2 >= 0 && w0 + w1 + w2 <= ldc, "amx_cost_rows: widths %d+%d+%d > ldc=%d", w0,
                w1, w2, ldc);
  AMX_CHECK_ARG((w0 == 0 || (x0 && ld0 >= w0)) && (w1 == 0 || (x1 && ld1 >= w1)) && (w2 == 0 || (x2 && ld2 >= w2)),
                "amx_cost_rows: missing segment or short row stride");
  if (B == 0) return AMX_OK;
  hipLaunchKernelGGL(k_cost_rows, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, x0, ld0, w0, x1, ld1, w1, x2,
                     ld2, w2, B, out, ldc);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_feature_message(amx_ctx* ctx, const double* partials, int n_parts, int F, double count,
                                   double* out, void* stream) {
  AMX_CHECK_ARG(ctx && partials && out && n_parts >= 0 && F > 0 && count >= 0.0, "amx_feature_message: bad argument");
  hipLaunchKernelGGL(k_feature_message, dim3((F + CS_COLS - 1) / CS_COLS), dim3(1024), 0, (hipStream_t)stream,
                     partials, n_parts, F, count, out);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_mmd_relabel(amx_ctx* ctx, const double* msg, double count, const float* phi_e, int F, float* w,
                               float* mmd, const float* phi, int ldphi, const float* disc, float thr, double lambda_b,
                               int clamp, float c_min, float c_max, float* reward, float* ipm, float* wbonus, int n,
                               const float* expert_rows, int ld_e, int n_e, double* expert_out, float* expert_mean,
                               uint32_t* counter, void* stream) {
  AMX_CHECK_ARG(ctx && msg && phi_e && w && mmd, "amx_mmd_relabel: null pointer");
  AMX_CHECK_ARG(F > 0 && F % 256 == 0 && F <= 4096, "amx_mmd_relabel: F=%d (multiple of 256, <= 4096)", F);
  AMX_CHECK_ARG(count >= 0.0, "amx_mmd_relabel: count=%g (0: read msg[F])", count);
  AMX_CHECK_ARG(n >= 0 && (n == 0 || (phi && disc && reward && ldphi >= F && ldphi % 4 == 0 && amx::aligned16(phi))),
                "amx_mmd_relabel: rollout rows n=%d need phi/disc/reward, ldphi=%d", n, ldphi);
  AMX_CHECK_ARG(expert_rows == nullptr || (clamp && n_e > 0 && ld_e >= F && ld_e % 4 == 0 && expert_out && counter &&
                                           amx::aligned16(expert_rows)),
                "amx_mmd_relabel: the expert cost needs clamp, n_e > 0, ld_e >= F, expert_out and counter");
  RelabelArgs a;
  a.msg = msg; a.count = count; a.phi_e = phi_e; a.F = F; a.w = w; a.mmd = mmd;
  a.phi = phi; a.ldphi = ldphi; a.disc = disc; a.thr = thr;
  a.one_m_lambda = (float)(1.0 - lambda_b); a.lambda_b = (float)lambda_b; a.c_min = c_min; a.c_max = c_max;
  a.reward = reward; a.ipm = ipm; a.wb = wbonus; a.n = n;
  a.erows = expert_rows; a.lde = ld_e; a.ne_rows = expert_rows ? n_e : 0;
  a.ne = expert_rows ? expert_blocks(n_e) : 0;
  a.eout = expert_out; a.emean = expert_mean; a.escale = (float)(1.0 - lambda_b); a.counter = counter;
  const size_t lds = (size_t)F * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  // NC = F/256 chunks per lane for F <= 1024 (R rows per round trip), else the generic path
  const int nc = F <= 1024 ? F / 256 : 0;
#define AMX_RELABEL_CASE(NC)                                                                              \
  case NC: {                                                                                              \
    constexpr int R = relabel_rows<NC>();                                                                 \
    a.nr = (n + 4 * R - 1) / (4 * R);                                                                     \
    const int blocks = (a.nr + a.ne) > 0 ? a.nr + a.ne : 1;                                               \
    if (clamp) hipLaunchKernelGGL((k_mmd_relabel<true, NC>), dim3(blocks), dim3(256), lds, st, a);        \
    else hipLaunchKernelGGL((k_mmd_relabel<false, NC>), dim3(blocks), dim3(256), lds, st, a);             \
    break;                                                                                                \
  }
  switch (nc) {
    AMX_RELABEL_CASE(0) AMX_RELABEL_CASE(1) AMX_RELABEL_CASE(2) AMX_RELABEL_CASE(3) AMX_RELABEL_CASE(4)
    default: break;
  }
#undef AMX_RELABEL_CASE
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}
