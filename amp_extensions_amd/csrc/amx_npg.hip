// The NPG policy update on the device: the learner step that consumes the rollout in the
// reference's MILO loop (mjrl NPG.train_from_paths, mjrl/mjrl/algos/npg_cg.py:113-199).
//
// Policy: mjrl MLP (gaussian_mlp.py:7-155) — mean = W3 tanh(W2 tanh(W1 x + b1) + b2) + b3,
// a ~ N(mean, exp(log_std)^2); parameters packed in the reference's flat order
// (trainable_params: W1 [H1][S], b1, W2 [H2][H1], b2, W3 [A][H2], b3, log_std [A]).
//
// One pass kernel, three modes, each block owning a contiguous run of rows and writing one
// fp64 partial vector (fixed-order reduction afterwards: deterministic):
//   VPG  grad of mean(LR * adv) at new == old (batch_reinforce.py:58-62, npg_cg.py:66-86):
//        dmean = adv/N * z/sigma, dlog_std = adv/N * (z^2 - 1), z = (a - mean)/sigma;
//   FVP  the mean-parameter part of NPG.HVP (npg_cg.py:87-106): the Hessian of mean_kl
//        (gaussian_mlp.py:144-155) at new == old is J^T diag(2/(2 sigma^2 + 1e-8)) J / N for
//        the mean network; the JVP J v is propagated forward, then back-propagated (the
//        log_std block, a diagonal constant, and the damping are added by the caller);
//   EVAL mean(LR * adv) and mean_kl of new vs old parameters (surr_after, kl_old_new,
//        npg_cg.py:181-183).
// Hidden widths are fixed at 32 (MILO's actor_model_hidden, milo/milo/arguments.py:95).
//
// Layout (round 3): a block of 8 waves walks its rows in chunks of 32.  Every product is a
// 16x16 tile on the f32 matrix pipe (v_mfma_f32_16x16x4_f32, an exact f32 fma chain):
//   * forward layer 1 (K = S, most of the flops): wave w owns the tile (units 16 (w & 1),
//     parameter set (w >> 1) % sets, rows 16 of the chunk) and keeps that tile's W1 (or tangent
//     V1) rows in registers for the whole kernel (staged once through LDS; kernels are compiled
//     for ceil(S / 16) rounded to 4 / 8 / 13 / 16 K-steps, so no MFMA sits under a branch); the
//     chunk's observations are the only K-long operand in LDS, read as float4s;
//   * layers 2 / 3 and the back-propagated deltas are 16x16 tiles over K = 32 / A, dealt
//     over the waves; the tanh derivative of a JVP is applied as its operand is loaded;
//   * the weight gradients (K = the chunk's rows) are tiles each wave owns across chunks,
//     accumulated on the matrix pipe in fp32 over the block's rows (fp64 across blocks in
//     amx_npg_reduce); the bias gradients come out of the same tiles through a column of ones
//     next to the layer's input (x[S] = 1, h[32] = 1: grad b = sum_r delta_r * 1);
//   * the next chunk's observations / actions / advantages are loaded into registers while
//     the current chunk computes, across LDS-only barriers.
// Round 2's kernel (scalar LDS FMA loops, 4 waves, 1 chunk-sum per thread) took 431 us per
// FVP pass at 40960 x 197; this one 60 ('The NPG learner').
#include "amx_common.h"

#include <type_traits>

// Phase mask for timing experiments (tools/npg_phase.py builds variants with -DNPG_PHASES=m):
// 1 layer 1, 2 layer 2, 4 output layer, 8 / 16 / 32 back-propagation of layers 3 / 2 / 1,
// 64 the chunk loads.  The library is always built with every phase.
#ifndef NPG_PHASES
#define NPG_PHASES 0x7f
#endif
// -DNPG_TRACE (tools/npg_phase.py trace): thread 0 of blocks 0, 64, 128, 255 stamps the device
// realtime clock (100 MHz) at the kernel's phase boundaries into npg_trace_buf.
#ifdef NPG_TRACE
__device__ unsigned long long npg_trace_buf[4][64];
#define NPG_STAMP(slot)                                                                        \
  do {                                                                                         \
    const int tb_ = blockIdx.x == 0 ? 0 : blockIdx.x == 64 ? 1 : blockIdx.x == 128 ? 2 : blockIdx.x == 255 ? 3 : -1; \
    if (threadIdx.x == 0 && tb_ >= 0 && (slot) < 64) npg_trace_buf[tb_][(slot)] = wall_clock64();   \
  } while (0)
#else
#define NPG_STAMP(slot) \
  do {                  \
  } while (0)
#endif

namespace {

constexpr int NH = 32;                 // hidden width (both layers)
constexpr int RC0 = 32;                // rows per chunk (64-row chunks measured slower: DESIGN.md section 6)
constexpr int NT = 512;                // threads per block: 8 waves, 2 per SIMD
constexpr int NW = NT / 64;
constexpr int MAXS = 256;              // max state dim
constexpr int MAXA = 64;               // max action dim
constexpr int HS = 52;                 // H1/H2 row stride: 32 units | 1 (ones column) | 0 to 48 | pad
constexpr int DS = 36;                 // D1/D2 (JVP, then delta) row stride
constexpr int WS = 36;                 // W2 / W3 LDS row stride
constexpr int MAXJJ = MAXS / 16;       // float4 W1 fragments per lane (at most)
constexpr int W1U = (NH * MAXS / 4 + NT - 1) / NT;  // W1 float4s per thread in the setup
constexpr int G1SLOTS = (2 * ((MAXS + 16) / 16) + NW - 1) / NW;  // gW1 tiles per wave
constexpr int G3SLOTS = (3 * (MAXA / 16) + NW - 1) / NW;         // gW3 tiles per wave

enum { NPG_VPG = 0, NPG_FVP = 1, NPG_EVAL = 2 };

// ---- conjugate gradient constants (cg_solve.py:3-23) ----
constexpr int CGT = 1024;
constexpr int CGE = 16;              // elements per thread: P <= CGT * CGE
constexpr int RCT = 1024, RCC = 64;  // k_npg_cg_reduce: threads, columns per block (16 run lanes per column)
constexpr int XRT = 1024;            // k_npg_cg_xrp threads (and elements owned) per block

// the sum of n fixed-order parts, computed the same way by every wave that calls it (lane-strided
// partial sums, then an xor butterfly: every lane ends with the same bits)
__device__ inline double parts_sum(const double* __restrict__ parts, int n) {
  const int lane = threadIdx.x & 63;
  double s = 0.0;
  for (int i = lane; i < n; i += 64) s += parts[i];
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) s += __shfl_xor(s, o);
  return s;
}


typedef float pf4 __attribute__((ext_vector_type(4)));

struct NpgArgs {
  int mode, N, S, A;
  int rows_per_block;
  const void* obs; long long ldo;
  const void* act; long long lda;
  const double* adv;         // VPG / EVAL (whitened advantages)
  const float* theta;        // packed parameters (old, for EVAL)
  const float* vec;          // FVP: tangent; EVAL: new parameters
  double* partials;          // VPG/FVP: [blocks][P]; EVAL: [blocks][2]
  int P;
  const double* gate;        // optional CG state {rdotr, live}: live == 0 -> the pass is a no-op
  float* hcache;             // optional theta forward [N][64] = H1 | H2: VPG writes it, FVP (HC) reads it
  // FVP with the previous CG iteration's vector step folded in (amx_npg_pass_cg; cg_state_in
  // null: the tangent is vec): the k_npg_cg_xrp operands, p' (not vec) is the tangent
  const double* cg_state_in; double* cg_state_out; double cg_tol;
  double* cg_x; const double* cg_r_in; double* cg_r_out;
  const double* cg_p_in; double* cg_p_out; float* cg_p32_out;
  const double* cg_work;     // k_npg_cg_reduce's output: z [P] | p.z parts
};
constexpr int HCW = 2 * 32;  // floats per cached row (H1 | H2)

struct Lay {  // offsets into the packed parameter vector
  int w1, b1, w2, b2, w3, b3, ls;
  __device__ Lay(int S, int A) {
    w1 = 0; b1 = NH * S; w2 = b1 + NH; b2 = w2 + NH * NH; w3 = b2 + NH; b3 = w3 + A * NH; ls = b3 + A;
  }
};

__host__ __device__ inline int npg_stride(int k) {  // LDS row stride (floats) of a [*][k] tile
  const int r = (k + 3) & ~3;
  return (r % 8 == 0) ? r + 4 : r;
}

struct Geo {
  int S, A, A16, nA, SW, nS, XS, GS, JJ;
  __host__ __device__ Geo(int S_, int A_) : S(S_), A(A_) {
    A16 = (A + 15) & ~15;
    nA = A16 / 16;
    SW = (S + 16) & ~15;   // gW1 columns: S inputs, the ones column (-> b1), zeros to 16
    nS = SW / 16;
    XS = npg_stride(SW);
    GS = npg_stride(A16);
    JJ = (S + 15) / 16;    // layer-1 K steps of 16 (one float4 per lane each)
  }
};

// LDS image of one parameter set's small part (W1 lives in registers)
struct Small {
  float *w2, *b2, *w3, *b3, *b1, *ls;
};

__host__ __device__ inline int r4(int n) { return (n + 3) & ~3; }

__host__ __device__ inline int small_floats(const Geo& g) {
  return r4(NH * WS) + r4(NH) + r4(g.A16 * WS) + r4(g.A16) + r4(NH) + r4(g.A16);
}

__device__ inline float* carve(float*& p, int n) {
  float* r = p;
  p += r4(n);
  return r;
}

__device__ inline Small carve_small(float*& p, const Geo& g) {
  Small s;
  s.w2 = carve(p, NH * WS); s.b2 = carve(p, NH); s.w3 = carve(p, g.A16 * WS);
  s.b3 = carve(p, g.A16); s.b1 = carve(p, NH); s.ls = carve(p, g.A16);
  return s;
}

// The small image as one flat index space: W2 [32][32] | W3 [A16][32] | b1 | b2 | b3 [A16] |
// ls [A16].  small_src: the packed-parameter index of element e (-1: a zero pad row);
// small_dst: its offset in the LDS image (carve_small's layout).
constexpr int SMU = (NH * NH + MAXA * NH + 2 * NH + 2 * MAXA + NT - 1) / NT;  // elements per thread

__host__ __device__ inline int small_count(const Geo& g) { return NH * NH + g.A16 * NH + 2 * NH + 2 * g.A16; }

__device__ inline int small_src(int e, const Lay& L, const Geo& g) {
  if (e < NH * NH) return L.w2 + e;
  e -= NH * NH;
  if (e < g.A16 * NH) return (e >> 5) < g.A ? L.w3 + e : -1;
  e -= g.A16 * NH;
  if (e < NH) return L.b1 + e;
  e -= NH;
  if (e < NH) return L.b2 + e;
  e -= NH;
  if (e < g.A16) return e < g.A ? L.b3 + e : -1;
  e -= g.A16;
  return e < g.A ? L.ls + e : -1;
}

__device__ inline int small_dst(int e, const Geo& g) {  // offsets as carve_small: w2, b2, w3, b3, b1, ls
  const int o_b2 = r4(NH * WS), o_w3 = o_b2 + r4(NH), o_b3 = o_w3 + r4(g.A16 * WS), o_b1 = o_b3 + r4(g.A16),
            o_ls = o_b1 + r4(NH);
  if (e < NH * NH) return (e >> 5) * WS + (e & 31);
  e -= NH * NH;
  if (e < g.A16 * NH) return o_w3 + (e >> 5) * WS + (e & 31);
  e -= g.A16 * NH;
  if (e < NH) return o_b1 + e;
  e -= NH;
  if (e < NH) return o_b2 + e;
  e -= NH;
  if (e < g.A16) return o_b3 + e;
  e -= g.A16;
  return o_ls + e;
}

// Workgroup barrier for LDS hand-offs: waits for this wave's LDS traffic only, so the next
// chunk's global loads stay in flight across it (__syncthreads' fence waits for them too).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// The CG fold (amx_npg_pass_cg): the previous iteration's vector step -- k_npg_cg_xrp's
// arithmetic in its orders, so the same bits -- at the head of the next Fisher-vector pass,
// which drops that launch from every iteration but the last.  Every block forms v = r.r / p.z
// from the p.z parts, r' = r - v z for all P elements and r'.r' in xrp's order (thread t
// stands in for xrp's threads t and t + 512: elements t + 512 k, k even / odd, two wave
// butterflies, the 16 wave sums in order), mu = r'.r' / r.r, and stages p' = r' + mu p as
// float32 in LDS (pb: P floats, then 16 doubles) for the tangent's parameter images; it writes
// its own slice of x += v p, r', p', float32(p') and block 0 the state {r'.r', live}.  Returns
// false when the solve has stopped (earlier, or now: r'.r' < tol): no product, as the gate.
__device__ __forceinline__ bool cg_fold(const NpgArgs& a, float* pb, int t) {
  const int P = a.P;
  const int cs = (P + gridDim.x - 1) / gridDim.x;
  const int lo = blockIdx.x * cs, hi = min(P, lo + cs);
  if (a.cg_state_in[1] == 0.0) {  // stopped: carry r and p over to the out buffers
    for (int e = lo + t; e < hi; e += NT) {
      const double pv = a.cg_p_in[e];
      a.cg_r_out[e] = a.cg_r_in[e];
      a.cg_p_out[e] = pv;
      a.cg_p32_out[e] = (float)pv;
    }
    if (blockIdx.x == 0 && t == 0) {
      a.cg_state_out[0] = a.cg_state_in[0];
      a.cg_state_out[1] = 0.0;
    }
    return false;
  }
  constexpr int K = 2 * CGE;  // P <= NT * K
  const double* zbuf = a.cg_work;
  double rl[K], zl[K], pl[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int e = t + NT * k;
    const bool ok = e < P;
    rl[k] = ok ? a.cg_r_in[e] : 0.0;
    zl[k] = ok ? zbuf[e] : 0.0;
    pl[k] = ok ? a.cg_p_in[e] : 0.0;
  }
  const double rdotr = a.cg_state_in[0];
  const double v = rdotr / parts_sum(zbuf + P, (P + RCC - 1) / RCC);
  double rr0 = 0.0, rr1 = 0.0;
#pragma unroll
  for (int u = 0; u < CGE; ++u) {
    rl[2 * u] = rl[2 * u] - v * zl[2 * u];
    rr0 += rl[2 * u] * rl[2 * u];
    rl[2 * u + 1] = rl[2 * u + 1] - v * zl[2 * u + 1];
    rr1 += rl[2 * u + 1] * rl[2 * u + 1];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    rr0 += __shfl_xor(rr0, o);
    rr1 += __shfl_xor(rr1, o);
  }
  double* red = reinterpret_cast<double*>(pb + r4(P));
  if ((t & 63) == 0) {
    red[t >> 6] = rr0;
    red[NW + (t >> 6)] = rr1;
  }
  lds_barrier();
  double rr = 0.0;
  for (int w = 0; w < 2 * NW; ++w) rr += red[w];
  const double mu = rr / rdotr;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int e = t + NT * k;
    if (e < P) {
      const double pn = rl[k] + mu * pl[k];
      pb[e] = (float)pn;
      if (e >= lo && e < hi) {
        a.cg_x[e] += v * pl[k];
        a.cg_r_out[e] = rl[k];
        a.cg_p_out[e] = pn;
        a.cg_p32_out[e] = (float)pn;
      }
    }
  }
  const bool live = !(rr < a.cg_tol);
  if (blockIdx.x == 0 && t == 0) {
    a.cg_state_out[0] = rr;
    a.cg_state_out[1] = live ? 1.0 : 0.0;
  }
  lds_barrier();  // p' staged
  return live;
}

__device__ __forceinline__ pf4 mma(float a, float b, pf4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int MODE, typename TO, typename TA, int RC, int JJM, bool HC = false>
__global__ __launch_bounds__(NT, 1) void k_npg(NpgArgs a) {
  // JJM: layer-1 K steps compiled (>= ceil(S / 16); steps past S multiply zero weights)
  // HC (FVP): the theta forward (H1, H2) is read from a.hcache, written by the VPG pass of the
  // same update (same kernels, same bits), instead of recomputed: layer 1 computes only the
  // tangent's tiles, its two MFMA chains (x.x/x.z and x.y/x.w) on two waves each, and layer 2's
  // two products of the tangent (H1 V2^T and D1' W2^T) on two waves -- every sum in the order
  // of the uncached pass, so the products are bit-identical to it
  constexpr int mode = MODE;
  constexpr bool HCF = HC && MODE == NPG_FVP;
  constexpr int NRB = RC / 16;                 // 16-row blocks per chunk
  constexpr int TPR = NT / RC;                 // staging threads per row
  constexpr int XU = MAXS / TPR, AU = MAXA / TPR;
  constexpr bool two = mode != NPG_VPG;
  constexpr int NMAT = two ? 2 : 1;            // parameter sets in the forward
  constexpr int NI = NRB * 2 * NMAT;           // layer-1 / layer-2 tiles per chunk
  constexpr int MI = (NI + NW - 1) / NW;       // ... per wave
  extern __shared__ __attribute__((aligned(16))) float sm[];
  if (a.gate && a.gate[1] == 0.0) return;  // CG has stopped (cg_solve.py:19-20): no product needed
  const Geo g(a.S, a.A);
  const Lay L(a.S, a.A);
  const int S = g.S, A = g.A;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, i = lane & 15, kq = lane >> 4;
  float* p = sm;
  const Small th = carve_small(p, g);
  Small tv = th;
  if (two) tv = carve_small(p, g);
  float* X = carve(p, RC * g.XS);     // [RC][XS]: S observations | 1 | zeros
  float* H1 = carve(p, RC * HS);      // tanh activations | 1 | zeros
  float* H2 = carve(p, RC * HS);
  float* D1 = carve(p, RC * DS);      // FVP: tangent pre-activation (V1 x + vb1); EVAL: new h1; then delta
  float* D2 = carve(p, RC * DS);
  float* G = carve(p, RC * g.GS);     // output-layer gradient (VPG / FVP), new mean (EVAL)
  float* M = mode == NPG_FVP ? G : carve(p, RC * g.GS);  // mean (EVAL), z (VPG)
  float* ACT = mode == NPG_FVP ? G : carve(p, RC * A);
  double* ADV = reinterpret_cast<double*>(mode == NPG_FVP ? G : carve(p, 2 * RC));
  float* TAB = carve(p, 2 * g.A16);   // per action: FVP 2 / (2 sigma^2 + 1e-8); VPG sigma; EVAL sigma_old | sigma_new

  NPG_STAMP(0);
  // FVP with the CG fold: the tangent p' is staged in LDS from the X tile on (read below, before
  // the W1 fragments reuse that space)
  bool fold = false;
  if constexpr (MODE == NPG_FVP) {
    if (a.cg_state_in) {
      if (!cg_fold(a, X, t)) return;
      fold = true;
    }
  }
  // Setup issues every global load before the first store (one memory round trip, not one per
  // array): W1 (and the tangent's / new W1) as coalesced float4s, the small parameter images,
  // the log_std table and the first chunk's inputs.  W1 then goes through LDS (the X tile's
  // space, before the first chunk) into each wave's fragment registers: read from global
  // memory directly, the fragments' row-strided lanes cost ~3 us of L1 line traffic.
  // Layer-1/2 tiles of this wave: item = wave + 8 m (m < MI): units 16 cb1, parameter set mat1
  // (the same for every m), rows 16 rb(m).
  const bool f1 = wave < NI;
  const int cb1 = wave & 1, mat1 = (wave >> 1) % NMAT;
  const int nw4 = NH * S / 4;  // float4s of W1 (32 S floats)
  pf4 w1a[W1U], w1b[W1U];
#pragma unroll
  for (int u = 0; u < W1U; ++u) {
    const int e = t + u * NT;
    w1a[u] = w1b[u] = pf4{0.f, 0.f, 0.f, 0.f};
    if (e < nw4) {
      if (!HCF) w1a[u] = reinterpret_cast<const pf4*>(a.theta)[e];
      if (two) w1b[u] = fold ? reinterpret_cast<const pf4*>(X)[e] : reinterpret_cast<const pf4*>(a.vec)[e];
    }
  }
  NPG_STAMP(50);
  const int nsmall = small_count(g);
  float sv0[SMU], sv1[SMU];
#pragma unroll
  for (int u = 0; u < SMU; ++u) {
    const int e = t + u * NT;
    sv0[u] = sv1[u] = 0.f;
    if (e < nsmall) {
      const int src = small_src(e, L, g);
      if (src >= 0) {
        sv0[u] = a.theta[src];
        if (two) sv1[u] = fold ? X[src] : a.vec[src];
      }
    }
  }
  NPG_STAMP(51);
  float lso = 0.f, lsn = 0.f;
  if (t < A) {
    lso = a.theta[L.ls + t];
    if (mode == NPG_EVAL) lsn = a.vec[L.ls + t];
  }

  // next chunk's inputs, held in registers while the current chunk computes: thread t stages
  // row t / TPR, columns t % TPR + TPR u (affine in u: one address register per array)
  TO xv[XU];
  TA av[AU];
  double dv = 0.0;
  pf4 hv = {0.f, 0.f, 0.f, 0.f};  // HC: cached row t / 16, floats 4 (t % 16) .. + 3
  const int pr = t / TPR, pc = t % TPR;
  constexpr bool need_act = mode != NPG_FVP;
  auto prefetch = [&](int c0, int nr) {
    const bool rv = pr < nr;
    const TO* xs = static_cast<const TO*>(a.obs) + (long long)(c0 + (rv ? pr : 0)) * a.ldo + pc;
#pragma unroll
    for (int u = 0; u < XU; ++u) xv[u] = (rv && pc + TPR * u < S) ? xs[TPR * u] : TO(0);
    if (need_act) {
      const TA* as = static_cast<const TA*>(a.act) + (long long)(c0 + (rv ? pr : 0)) * a.lda + pc;
#pragma unroll
      for (int u = 0; u < AU; ++u) av[u] = (rv && pc + TPR * u < A) ? as[TPR * u] : TA(0);
      if (t < RC) dv = t < nr ? a.adv[c0 + t] : 0.0;
    }
    if (HCF) {
      const int hr = t >> 4;
      hv = (t < RC * 16 && hr < nr) ? *reinterpret_cast<const pf4*>(a.hcache + (long long)(c0 + hr) * HCW + 4 * (t & 15))
                                     : pf4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto stash = [&]() {
    float* xd = X + pr * g.XS + pc;
#pragma unroll
    for (int u = 0; u < XU; ++u)
      if (pc + TPR * u < S) xd[TPR * u] = (float)xv[u];  // np.float32(observation)
    if (need_act) {
      float* ad = ACT + pr * A + pc;
#pragma unroll
      for (int u = 0; u < AU; ++u)
        if (pc + TPR * u < A) ad[TPR * u] = (float)av[u];
      if (t < RC) ADV[t] = dv;
    }
    if (HCF && t < RC * 16) {
      const int hr = t >> 4, hc = t & 15;
      *reinterpret_cast<pf4*>((hc < 8 ? H1 + 4 * hc : H2 + 4 * (hc - 8)) + hr * HS) = hv;
    }
  };
  const int r0 = blockIdx.x * a.rows_per_block;
  const int r1 = min(a.N, r0 + a.rows_per_block);
  NPG_STAMP(52);
  if (r0 < r1) prefetch(r0, min(RC, r1 - r0));
  NPG_STAMP(53);
  if (fold) lds_barrier();  // every wave has read p' before the fragments overwrite X

  // W1 fragments via LDS: set 0, then (FVP / EVAL) set 1, through the X tile's space
  pf4 wf[JJM];
  auto fragments = [&](const pf4 (&w)[W1U], int set) {
#pragma unroll
    for (int u = 0; u < W1U; ++u) {
      const int e = t + u * NT;
      if (e < nw4) reinterpret_cast<pf4*>(X)[e] = w[u];
    }
    lds_barrier();
    if (f1 && (mat1 == set || HCF)) {  // HC: every wave holds the tangent's W1 rows
      const float* wrow = X + (cb1 * 16 + i) * S;
#pragma unroll
      for (int jj = 0; jj < JJM; ++jj) {
        pf4 v = {0.f, 0.f, 0.f, 0.f};
        const int k0 = 4 * (kq + 4 * jj);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (k0 + e < S) v[e] = wrow[k0 + e];
        wf[jj] = v;
      }
    }
    lds_barrier();
  };
#pragma unroll
  for (int jj = 0; jj < JJM; ++jj) wf[jj] = pf4{0.f, 0.f, 0.f, 0.f};
  if (!HCF) fragments(w1a, 0);
  if (two) fragments(w1b, 1);

  // stores: parameter images, constant pads, the per-action table
#pragma unroll
  for (int u = 0; u < SMU; ++u) {
    const int e = t + u * NT;
    if (e < nsmall) {
      const int o = small_dst(e, g);
      sm[o] = sv0[u];
      if (two) sm[small_floats(g) + o] = sv1[u];
    }
  }
  {
    const int xp = g.XS - S;
    for (int e = t; e < RC * xp; e += NT) {
      const int r = e / xp, c = S + e % xp;
      X[r * g.XS + c] = c == S ? 1.f : 0.f;
    }
    for (int e = t; e < RC * (HS - NH); e += NT) {
      const int r = e / (HS - NH), c = NH + e % (HS - NH);
      H1[r * HS + c] = c == NH ? 1.f : 0.f;
      H2[r * HS + c] = c == NH ? 1.f : 0.f;
    }
    if (t < g.A16) {
      const float sd = t < A ? expf(lso) : 1.f;
      TAB[t] = mode == NPG_FVP ? 2.f / (2.f * sd * sd + 1e-8f) : sd;
      if (mode == NPG_EVAL) TAB[g.A16 + t] = t < A ? expf(lsn) : 1.f;
    }
  }
  NPG_STAMP(54);

  NPG_STAMP(55);
  // the owned weight-gradient tiles: MFMA accumulators carried across the block's chunks
  // (fp32 over the block's rows, fp64 across blocks in amx_npg_reduce)
  pf4 g1[G1SLOTS], g3[G3SLOTS], g2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < G1SLOTS; ++s) g1[s] = pf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < G3SLOTS; ++s) g3[s] = pf4{0.f, 0.f, 0.f, 0.f};
  double gls = 0.0, ev_surr = 0.0, ev_kl = 0.0;
  const double invN = 1.0 / (double)a.N;

  for (int c0 = r0, ci = 0; c0 < r1; c0 += RC, ++ci) {
    // per-chunk opaque copies of the lane indices and strides: keeps the compiler from hoisting
    // every chunk-invariant LDS address out of the loop (hundreds of registers held live)
    int i_ = i, kq_ = kq, xs_ = g.XS, gs_ = g.GS, jj_ = g.JJ;
    asm volatile("" : "+v"(i_), "+v"(kq_));
    asm volatile("" : "+s"(xs_), "+s"(gs_), "+s"(jj_));
    const int i = i_, kq = kq_, XS = xs_, GS = gs_, JJ = jj_;
    const int nr = min(RC, r1 - c0);
    lds_barrier();  // the previous chunk is consumed (first chunk: parameters and pads are stored)
    NPG_STAMP(2 + 8 * ci + 0);
    if (NPG_PHASES & 64) {
      stash();
      if (c0 + RC < r1) prefetch(c0 + RC, min(RC, r1 - c0 - RC));
    }
    lds_barrier();
    NPG_STAMP(2 + 8 * ci + 1);

    // ---- layer 1: H1 = tanh(X W1^T + b1); FVP: D1 = X V1^T + vb1; EVAL: D1 = tanh(X V1n^T + b1n)
    if constexpr (HCF) {
      // the tangent's 4 tiles (units 16 cb, rows 16 rb), each as two chains: waves with
      // (wave >> 1) & 1 == 0 the x.x / x.z chain (ca), the others the x.y / x.w chain (cb),
      // which they leave in D1; then z = (ca + cb) + vb1 as the uncached pass forms it
      if (NPG_PHASES & 1) {
        const int cb = wave & 1, rb = wave >> 2, ch = (wave >> 1) & 1;
        const float* xr = X + (rb * 16 + i) * XS + 4 * kq;
        pf4 acc = {0.f, 0.f, 0.f, 0.f};
        pf4 xq[2];
        xq[0] = *reinterpret_cast<const pf4*>(xr);
        xq[1] = *reinterpret_cast<const pf4*>(xr + 16 * min(1, JJ - 1));
        if (ch == 0) {
#pragma unroll
          for (int jj = 0; jj < JJM; ++jj) {
            const pf4 x = xq[jj & 1];
            if (jj + 2 < JJM) xq[jj & 1] = *reinterpret_cast<const pf4*>(xr + 16 * min(jj + 2, JJ - 1));
            acc = mma(x.x, wf[jj].x, acc);
            acc = mma(x.z, wf[jj].z, acc);
          }
        } else {
#pragma unroll
          for (int jj = 0; jj < JJM; ++jj) {
            const pf4 x = xq[jj & 1];
            if (jj + 2 < JJM) xq[jj & 1] = *reinterpret_cast<const pf4*>(xr + 16 * min(jj + 2, JJ - 1));
            acc = mma(x.y, wf[jj].y, acc);
            acc = mma(x.w, wf[jj].w, acc);
          }
        }
        const int col = cb * 16 + i;
        if (ch) {
#pragma unroll
          for (int r = 0; r < 4; ++r) D1[(rb * 16 + 4 * kq + r) * DS + col] = acc[r];
        }
        lds_barrier();
        if (!ch) {
          const float bias = tv.b1[col];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* d = D1 + (rb * 16 + 4 * kq + r) * DS + col;
            *d = (acc[r] + *d) + bias;
          }
        }
      }
    } else if ((NPG_PHASES & 1) && f1) {
      const float* xr[MI];
      pf4 ca[MI], cb[MI], xq[MI][2];
#pragma unroll
      for (int m = 0; m < MI; ++m) {
        xr[m] = X + (((wave + NW * m) / (2 * NMAT)) * 16 + i) * XS + 4 * kq;
        ca[m] = cb[m] = pf4{0.f, 0.f, 0.f, 0.f};
        // software-pipelined: step jj + 2's operand is read while step jj multiplies (clamped to
        // the last step: a read past JJ is never used)
        xq[m][0] = *reinterpret_cast<const pf4*>(xr[m]);
        xq[m][1] = *reinterpret_cast<const pf4*>(xr[m] + 16 * min(1, JJ - 1));
      }
#pragma unroll
      for (int jj = 0; jj < JJM; ++jj) {  // no branch: a guarded MFMA costs accumulator copies
        pf4 x[MI];
#pragma unroll
        for (int m = 0; m < MI; ++m) {
          x[m] = xq[m][jj & 1];
          if (jj + 2 < JJM) xq[m][jj & 1] = *reinterpret_cast<const pf4*>(xr[m] + 16 * min(jj + 2, JJ - 1));
        }
#pragma unroll
        for (int m = 0; m < MI; ++m) {
          ca[m] = mma(x[m].x, wf[jj].x, ca[m]);
          cb[m] = mma(x[m].y, wf[jj].y, cb[m]);
          ca[m] = mma(x[m].z, wf[jj].z, ca[m]);
          cb[m] = mma(x[m].w, wf[jj].w, cb[m]);
        }
      }
      const int col = cb1 * 16 + i;
      const float bias = (mat1 ? tv.b1 : th.b1)[col];
#pragma unroll
      for (int m = 0; m < MI; ++m) {
        const int rb = (wave + NW * m) / (2 * NMAT);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rb * 16 + 4 * kq + r;
          const float z = (ca[m][r] + cb[m][r]) + bias;
          if (!mat1) {
            const float hz = tanhf(z);
            H1[row * HS + col] = hz;
            if (mode == NPG_VPG && a.hcache && row < nr) a.hcache[(long long)(c0 + row) * HCW + col] = hz;
          } else {
            D1[row * DS + col] = mode == NPG_EVAL ? tanhf(z) : z;  // FVP: tanh' applied on use
          }
        }
      }
    }
    lds_barrier();
    NPG_STAMP(2 + 8 * ci + 2);

    // ---- layer 2 (the layer-1 tiles): H2 = tanh(H1 W2^T + b2);
    //      FVP: D2 = H1 V2^T + (D1 (1 - H1^2)) W2^T + vb2; EVAL: D2 = tanh(D1 V2n^T + b2n)
    if constexpr (HCF) {
      // the tangent's two products on two waves per tile: (wave >> 1) & 1 == 0 the D1' W2^T
      // term (left in D2), the others H1 V2^T, then D2 = (H1 V2^T + D1' W2^T) + vb2
      if (NPG_PHASES & 2) {
        const int u = (wave & 1) * 16 + i, rb = wave >> 2, ch = (wave >> 1) & 1;
        const int rowA = rb * 16 + i;
        pf4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < NH / 4; ++s2) {
          const int k = 4 * s2 + kq;
          const float h = H1[rowA * HS + k];
          if (ch) acc = mma(h, tv.w2[u * WS + k], acc);
          else acc = mma(D1[rowA * DS + k] * (1.f - h * h), th.w2[u * WS + k], acc);
        }
        if (!ch) {  // (D2 is not read in this phase: its last readers are behind earlier barriers)
#pragma unroll
          for (int r = 0; r < 4; ++r) D2[(rb * 16 + 4 * kq + r) * DS + u] = acc[r];
        }
        lds_barrier();
        if (ch) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* d = D2 + (rb * 16 + 4 * kq + r) * DS + u;
            *d = (acc[r] + *d) + tv.b2[u];
          }
        }
      }
    } else if ((NPG_PHASES & 2) && f1) {
      const int u = cb1 * 16 + i;
      pf4 acc[MI], acc2[MI];
#pragma unroll
      for (int m = 0; m < MI; ++m) acc[m] = acc2[m] = pf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NH / 4; ++s) {
        const int k = 4 * s + kq;
#pragma unroll
        for (int m = 0; m < MI; ++m) {
          const int rowA = ((wave + NW * m) / (2 * NMAT)) * 16 + i;
          if (!mat1) {
            acc[m] = mma(H1[rowA * HS + k], th.w2[u * WS + k], acc[m]);
          } else if (mode == NPG_FVP) {
            const float h = H1[rowA * HS + k];
            acc[m] = mma(h, tv.w2[u * WS + k], acc[m]);
            acc2[m] = mma(D1[rowA * DS + k] * (1.f - h * h), th.w2[u * WS + k], acc2[m]);
          } else {
            acc[m] = mma(D1[rowA * DS + k], tv.w2[u * WS + k], acc[m]);
          }
        }
      }
#pragma unroll
      for (int m = 0; m < MI; ++m) {
        const int rb = (wave + NW * m) / (2 * NMAT);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rb * 16 + 4 * kq + r;
          if (!mat1) {
            const float hz = tanhf(acc[m][r] + th.b2[u]);
            H2[row * HS + u] = hz;
            if (mode == NPG_VPG && a.hcache && row < nr) a.hcache[(long long)(c0 + row) * HCW + NH + u] = hz;
          }
          else if (mode == NPG_FVP) D2[row * DS + u] = (acc[m][r] + acc2[m][r]) + tv.b2[u];
          else D2[row * DS + u] = tanhf(acc[m][r] + tv.b2[u]);
        }
      }
    }
    lds_barrier();
    NPG_STAMP(2 + 8 * ci + 3);

    // ---- output layer: VPG mean -> G (and z -> M); FVP JVP of the mean -> G; EVAL M, new mean G
    if (NPG_PHASES & 4) {
      const int n3 = NRB * g.nA * (mode == NPG_EVAL ? 2 : 1);
      for (int it = wave; it < n3; it += NW) {
        const int rb = it % NRB, cbk = (it / NRB) % g.nA, mat = it / (NRB * g.nA);
        const int rowA = rb * 16 + i, u = cbk * 16 + i;
        pf4 acc = {0.f, 0.f, 0.f, 0.f}, acc2 = {0.f, 0.f, 0.f, 0.f};
        if (mode == NPG_FVP) {
#pragma unroll
          for (int s = 0; s < NH / 4; ++s) {
            const int k = 4 * s + kq;
            const float h = H2[rowA * HS + k];
            acc = mma(h, tv.w3[u * WS + k], acc);
            acc2 = mma(D2[rowA * DS + k] * (1.f - h * h), th.w3[u * WS + k], acc2);
          }
        } else if (!mat) {
#pragma unroll
          for (int s = 0; s < NH / 4; ++s) {
            const int k = 4 * s + kq;
            acc = mma(H2[rowA * HS + k], th.w3[u * WS + k], acc);
          }
        } else {
#pragma unroll
          for (int s = 0; s < NH / 4; ++s) {
            const int k = 4 * s + kq;
            acc = mma(D2[rowA * DS + k], tv.w3[u * WS + k], acc);
          }
        }
        const int d = u;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rb * 16 + 4 * kq + r;
          const bool ok = row < nr && d < A;
          if (mode == NPG_FVP) {
            const float m = (acc[r] + acc2[r]) + tv.b3[d];
            G[row * GS + d] = ok ? (float)((double)(m * TAB[d]) * invN) : 0.f;
          } else if (mode == NPG_VPG) {
            const float m = acc[r] + th.b3[d];
            float gg = 0.f, z = 0.f;
            if (ok) {
              const float sd = TAB[d];
              z = (ACT[row * A + d] - m) / sd;
              gg = (float)(ADV[row] * invN) * (z / sd);
            }
            G[row * GS + d] = gg;
            M[row * GS + d] = z;
          } else {
            (mat ? G : M)[row * GS + d] = acc[r] + (mat ? tv.b3 : th.b3)[d];
          }
        }
      }
    }
    lds_barrier();
    NPG_STAMP(2 + 8 * ci + 4);

    if (mode == NPG_EVAL) {
      // per row: LL_new - LL_old and sample_kl (gaussian_mlp.py:110-155); TPR threads per row
      // (actions pc + TPR u), combined over the TPR by butterfly shuffles
      float dll = 0.f, kl = 0.f;
      for (int d = pc; d < A; d += TPR) {
        const float ac = ACT[pr * A + d];
        const float mo = M[pr * GS + d], mn = G[pr * GS + d];
        const float so = TAB[d], sn = TAB[g.A16 + d];
        const float zo = (ac - mo) / so, zn = (ac - mn) / sn;
        dll += -0.5f * zn * zn - (-0.5f * zo * zo) + (th.ls[d] - tv.ls[d]);
        const float dm = mo - mn;
        const float Nr = dm * dm + so * so - sn * sn, Dr = 2.f * sn * sn + 1e-8f;
        kl += Nr / Dr + tv.ls[d] - th.ls[d];
      }
#pragma unroll
      for (int o = 1; o < TPR; o <<= 1) {
        dll += __shfl_xor(dll, o);
        kl += __shfl_xor(kl, o);
      }
      if (pc == 0 && pr < nr) {
        ev_surr += (double)(expf(dll) * (float)ADV[pr]);
        ev_kl += (double)kl;
      }
      continue;
    }

    // ---- back-propagation, output layer: gW3 | b3 (owned tiles, K = rows);
    //      D2 = (G W3)(1 - H2^2) (tiles from the last wave down); VPG: log_std sums (wave 3)
    if (NPG_PHASES & 8) {
#pragma unroll
      for (int sl = 0; sl < G3SLOTS; ++sl) {
        const int q = wave + NW * sl;
        if (q < 3 * g.nA) {
          const int mb = q / 3, nb = q % 3;
          pf4 acc = g3[sl];
#pragma unroll
          for (int s = 0; s < RC / 4; ++s) {
            const int k = 4 * s + kq;
            acc = mma(G[k * GS + mb * 16 + i], H2[k * HS + nb * 16 + i], acc);
          }
          g3[sl] = acc;
        }
      }
      for (int it = NW - 1 - wave; it < 2 * NRB; it += NW) {
        const int rb = it % NRB, cbk = it / NRB;
        const int rowA = rb * 16 + i, col = cbk * 16 + i;
        pf4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int s = 0; s < g.A16 / 4; ++s) {
          const int k = 4 * s + kq;
          acc = mma(G[rowA * GS + k], th.w3[k * WS + col], acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rb * 16 + 4 * kq + r;
          const float h = H2[row * HS + col];
          D2[row * DS + col] = acc[r] * (1.f - h * h);
        }
      }
      if (mode == NPG_VPG && t >= 192 && t < 192 + A) {
        const int d = t - 192;
        for (int r = 0; r < nr; ++r) {
          const float z = M[r * GS + d];
          gls += ADV[r] * invN * (double)(z * z - 1.f);
        }
      }
    }
    lds_barrier();
    NPG_STAMP(2 + 8 * ci + 5);

    // ---- layer 2: gW2 | b2 (waves 0-5); D1 = (D2 W2)(1 - H1^2) (tiles from the last wave down)
    if (NPG_PHASES & 16) {
      if (wave < 6) {
        const int mb = wave / 3, nb = wave % 3;
        pf4 acc = g2;
#pragma unroll
        for (int s = 0; s < RC / 4; ++s) {
          const int k = 4 * s + kq;
          acc = mma(D2[k * DS + mb * 16 + i], H1[k * HS + nb * 16 + i], acc);
        }
        g2 = acc;
      }
      for (int it = NW - 1 - wave; it < 2 * NRB; it += NW) {
        const int rb = it % NRB, cbk = it / NRB;
        const int rowA = rb * 16 + i, col = cbk * 16 + i;
        pf4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < NH / 4; ++s) {
          const int k = 4 * s + kq;
          acc = mma(D2[rowA * DS + k], th.w2[k * WS + col], acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rb * 16 + 4 * kq + r;
          const float h = H1[row * HS + col];
          D1[row * DS + col] = acc[r] * (1.f - h * h);
        }
      }
    }
    lds_barrier();
    NPG_STAMP(2 + 8 * ci + 6);

    // ---- layer 1: gW1 | b1 (owned tiles q = wave + 8 sl: mb = wave & 1 for every slot, so the
    //      D1 operand is shared and the slots' chains interleave; the slot count is the block's
    //      ceil(2 nS / 8), a slot past this wave's tiles computes and is discarded)
    if (NPG_PHASES & 32) {
      auto bp1 = [&](auto nsl_c) {
        constexpr int NSL = decltype(nsl_c)::value;
        const int mb = wave & 1;
        pf4 acc[NSL];
#pragma unroll
        for (int sl = 0; sl < NSL; ++sl) acc[sl] = g1[sl];
#pragma unroll
        for (int s = 0; s < RC / 4; ++s) {
          const int k = 4 * s + kq;
          const float d = D1[k * DS + mb * 16 + i];
          float xb[NSL];
#pragma unroll
          for (int sl = 0; sl < NSL; ++sl) {
            const int nb = min((wave >> 1) + (NW / 2) * sl, g.nS - 1);
            xb[sl] = X[k * XS + nb * 16 + i];
          }
#pragma unroll
          for (int sl = 0; sl < NSL; ++sl) acc[sl] = mma(d, xb[sl], acc[sl]);
        }
#pragma unroll
        for (int sl = 0; sl < NSL; ++sl) g1[sl] = acc[sl];
      };
      switch ((2 * g.nS + NW - 1) / NW) {
        case 1: bp1(std::integral_constant<int, 1>{}); break;
        case 2: bp1(std::integral_constant<int, 2>{}); break;
        case 3: bp1(std::integral_constant<int, 3>{}); break;
        case 4: bp1(std::integral_constant<int, 4>{}); break;
        default: bp1(std::integral_constant<int, G1SLOTS>{}); break;
      }
    }
    NPG_STAMP(2 + 8 * ci + 7);
  }

  if (mode == NPG_EVAL) {
    // block sums of (surr, kl): fixed-order tree
    __syncthreads();
    double* red = reinterpret_cast<double*>(H1);  // the activation tiles are free now
    red[t] = ev_surr;
    red[NT + t] = ev_kl;
    __syncthreads();
    for (int h = NT / 2; h > 0; h >>= 1) {
      if (t < h) {
        red[t] += red[t + h];
        red[NT + t] += red[NT + t + h];
      }
      __syncthreads();
    }
    if (t == 0) {
      a.partials[2LL * blockIdx.x] = red[0];
      a.partials[2LL * blockIdx.x + 1] = red[NT];
    }
    return;
  }
  // tile element (row 16 mb + 4 kq + r, column 16 nb + i); the ones column is the bias
  NPG_STAMP(1);
  double* out = a.partials + (long long)blockIdx.x * a.P;
#pragma unroll
  for (int sl = 0; sl < G1SLOTS; ++sl) {
    const int q = wave + NW * sl;
    if (q < 2 * g.nS) {
      const int mb = q & 1, nb = q >> 1, k = nb * 16 + i;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = mb * 16 + 4 * kq + r;
        if (k < S) out[L.w1 + j * S + k] = (double)g1[sl][r];
        else if (k == S) out[L.b1 + j] = (double)g1[sl][r];
      }
    }
  }
  if (wave < 6) {
    const int mb = wave / 3, nb = wave % 3, k = nb * 16 + i;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = mb * 16 + 4 * kq + r;
      if (k < NH) out[L.w2 + j * NH + k] = (double)g2[r];
      else if (k == NH) out[L.b2 + j] = (double)g2[r];
    }
  }
#pragma unroll
  for (int sl = 0; sl < G3SLOTS; ++sl) {
    const int q = wave + NW * sl;
    if (q < 3 * g.nA) {
      const int mb = q / 3, nb = q % 3, k = nb * 16 + i;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int d = mb * 16 + 4 * kq + r;
        if (d < A) {
          if (k < NH) out[L.w3 + d * NH + k] = (double)g3[sl][r];
          else if (k == NH) out[L.b3 + d] = (double)g3[sl][r];
        }
      }
    }
  }
  if (t >= 192 && t < 192 + A) out[L.ls + t - 192] = mode == NPG_VPG ? gls : 0.0;
  NPG_STAMP(63);
}

// out[c] = sum_b partials[b][c] in a fixed order (deterministic): stage 1 sums runs of RB
// consecutive blocks per column (grid.y = run), stage 2 sums the runs in order.
constexpr int RB = 16;
__global__ void k_npg_reduce1(const double* __restrict__ part, int nb, int P, double* __restrict__ mid,
                              const double* __restrict__ gate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= P || (gate && gate[1] == 0.0)) return;
  const int b0 = blockIdx.y * RB, b1 = min(nb, b0 + RB);
  double s = 0.0;
#pragma unroll 8
  for (int b = b0; b < b1; ++b) s += part[(long long)b * P + c];  // 8 loads in flight, same add order
  mid[(long long)blockIdx.y * P + c] = s;
}
__global__ void k_npg_reduce2(const double* __restrict__ mid, int nr, int P, double* __restrict__ out,
                              const double* __restrict__ gate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= P || (gate && gate[1] == 0.0)) return;
  double s = 0.0;
#pragma unroll 8
  for (int r = 0; r < nr; ++r) s += mid[(long long)r * P + c];
  out[c] = s;
}

// ---- conjugate gradient (cg_solve.py:3-23) ---------------------------------------------
// sum over the workgroup in a fixed order (per-thread sums, wave butterflies, waves in order)
__device__ double cg_block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < CGT / 64; ++w) s += red[w];
  __syncthreads();  // red is reused by the next sum
  return s;
}

__device__ inline double npg_ls_curvature(float log_std) {
  const double e = exp((double)log_std);
  const double sq = e * e, eps = 1e-8;
  const double den = 2.0 * sq + eps;
  return (8.0 * sq * sq - 4.0 * sq * eps) / (den * den);
}

// (theta / curv non-null: also the log_std curvature of k_npg_curvature, one launch fewer)
__global__ __launch_bounds__(CGT) void k_npg_cg_init(int P, const double* __restrict__ b, double* __restrict__ x,
                                                     double* __restrict__ r, double* __restrict__ p,
                                                     float* __restrict__ p32, double* __restrict__ state, int A,
                                                     const float* __restrict__ theta, double* __restrict__ curv) {
  __shared__ double red[CGT / 64];
  if (curv)
    for (int d = threadIdx.x; d < A; d += CGT) curv[d] = npg_ls_curvature(theta[P - A + d]);
  double rr = 0.0;
#pragma unroll
  for (int u = 0; u < CGE; ++u) {
    const int e = threadIdx.x + u * CGT;
    if (e < P) {
      const double bv = b[e];
      x[e] = 0.0;
      r[e] = bv;
      p[e] = bv;
      p32[e] = (float)bv;
      rr += bv * bv;
    }
  }
  rr = cg_block_sum(rr, red);
  if (threadIdx.x == 0) {
    state[0] = rr;
    state[1] = 1.0;
  }
}

__global__ __launch_bounds__(CGT) void k_npg_cg_step(int P, int A, const double* __restrict__ h,
                                                     const double* __restrict__ curv, double damping, double tol,
                                                     double* __restrict__ x, double* __restrict__ r,
                                                     double* __restrict__ p, float* __restrict__ p32,
                                                     double* __restrict__ state) {
  __shared__ double red[CGT / 64];
  if (state[1] == 0.0) return;  // the solve has stopped (uniform)
  const double rdotr = state[0];
  double zl[CGE], pl[CGE], pz = 0.0;
#pragma unroll
  for (int u = 0; u < CGE; ++u) {
    const int e = threadIdx.x + u * CGT;
    zl[u] = pl[u] = 0.0;
    if (e < P) {
      const double pv = p[e];
      double z = h[e];
      if (e >= P - A) z += curv[e - (P - A)] * (double)p32[e];
      z += damping * pv;
      zl[u] = z;
      pl[u] = pv;
      pz += pv * z;
    }
  }
  pz = cg_block_sum(pz, red);
  const double v = rdotr / pz;
  double rl[CGE], rr = 0.0;
#pragma unroll
  for (int u = 0; u < CGE; ++u) {
    const int e = threadIdx.x + u * CGT;
    rl[u] = 0.0;
    if (e < P) {
      x[e] += v * pl[u];
      const double rv = r[e] - v * zl[u];
      r[e] = rv;
      rl[u] = rv;
      rr += rv * rv;
    }
  }
  rr = cg_block_sum(rr, red);
  const double mu = rr / rdotr;
#pragma unroll
  for (int u = 0; u < CGE; ++u) {
    const int e = threadIdx.x + u * CGT;
    if (e < P) {
      const double pn = rl[u] + mu * pl[u];
      p[e] = pn;
      p32[e] = (float)pn;
    }
  }
  if (threadIdx.x == 0) {
    state[0] = rr;
    state[1] = rr < tol ? 0.0 : 1.0;
  }
}

// d^2 mean_kl / d log_std^2 at new == old per action (gaussian_mlp.py:144-155 with Dr's 1e-8),
// in DeviceNPG._ls_curvature's operation order: s = exp(log_std)^2,
// (8 s s - 4 s eps) / (2 s + eps)^2
__global__ __launch_bounds__(64) void k_npg_curvature(const float* __restrict__ theta, int P, int A,
                                                      double* __restrict__ curv) {
  const int d = blockIdx.x * 64 + threadIdx.x;
  if (d >= A) return;
  curv[d] = npg_ls_curvature(theta[P - A + d]);
}

// The NPG step after the CG (npg_cg.py:141-163): gdot = vpg . npg (fixed-order block sum);
// const_learn_rate: alpha given, n_step_size = alpha^2 gdot; else n_step_size given,
// alpha = sqrt(|n_step_size / (gdot + 1e-20)|); new = float32(float64(theta) + alpha npg), its
// log_std block clamped below at min_log_std (gaussian_mlp.py:71-94; NaN stays NaN, as
// torch.clamp).  scal = {alpha, n_step_size, gdot}.
__global__ __launch_bounds__(CGT) void k_npg_apply(int P, int A, const double* __restrict__ vpg,
                                                   const double* __restrict__ npg, const float* __restrict__ theta,
                                                   int use_alpha, double alpha_in, double nss_in, float min_ls,
                                                   float* __restrict__ out, double* __restrict__ scal) {
  __shared__ double red[CGT / 64];
  double gl = 0.0;
#pragma unroll
  for (int u = 0; u < CGE; ++u) {
    const int e = threadIdx.x + u * CGT;
    if (e < P) gl += vpg[e] * npg[e];
  }
  const double gdot = cg_block_sum(gl, red);
  double alpha, nss;
  if (use_alpha) {
    alpha = alpha_in;
    nss = alpha * alpha * gdot;
  } else {
    nss = nss_in;
    alpha = sqrt(fabs(nss / (gdot + 1e-20)));
  }
#pragma unroll
  for (int u = 0; u < CGE; ++u) {
    const int e = threadIdx.x + u * CGT;
    if (e < P) {
      float v = (float)((double)theta[e] + alpha * npg[e]);
      if (e >= P - A && v < min_ls) v = min_ls;
      out[e] = v;
    }
  }
  if (threadIdx.x == 0) {
    scal[0] = alpha;
    scal[1] = nss;
    scal[2] = gdot;
  }
}

// One CG iteration's tail (amx_npg_reduce + amx_npg_cg_step's arithmetic) in two launches spread
// over the chip.  The round-4 form ran the whole vector step and the serial sum of the blocks'
// p.z parts in the last-arriving block (20 us per iteration: one CU moving 275 KB behind two
// agent-scope fences); every launch costs ~5 us even when tiny (k_npg_curvature, one 64-thread
// workgroup: 4.8 us under rocprofv3), so the tail is as few launches as its two grid-wide
// dependencies allow:
//  k_npg_cg_reduce: a 1024-thread block per 64 columns, one thread per (column, run of RB FVP
//    blocks) summing the run's rows, one thread per column adding the runs in order (the
//    amx_npg_reduce order: the same h bits); z = h + [curv p32] + damping p into zbuf and the
//    block's part of p.z (its columns in order) into pzp[block];
//  k_npg_cg_xrp: 1024 threads per block, each block owning 1024 elements.  Every wave sums the
//    p.z parts in the same fixed order (lane l: parts l, l + 64, ...; then a butterfly whose
//    association is the same in every lane), so every block has the same v = rdotr / p.z; every
//    block then forms r' = r - v z for ALL P elements and sums r'.r' in one fixed order (the same
//    bits in every block: mu = r'.r' / rdotr needs no second grid-wide step), and updates its own
//    elements: x += v p, r' into r_out, p = r' + mu p, p32.  Block 0 writes {r'.r', live} into
//    state_out.  r and the state alternate between two buffers (in -> out) because every block
//    reads all of r while the others write theirs; a stopped solve (state_in live == 0) only
//    carries r and the state over, so every later iteration stays stopped.
// work = [zbuf: P | pz parts: ceil(P / 64)].
// (RCT, RCC, XRT: with the CG constants at the top of the file)

__global__ __launch_bounds__(RCT) void k_npg_cg_reduce(const double* __restrict__ part, int nb, int P, int A,
                                                       const double* __restrict__ curv, double damping,
                                                       const double* __restrict__ p, const float* __restrict__ p32,
                                                       const double* __restrict__ state, double* __restrict__ work) {
  __shared__ double runs[RCT];  // [run][column]
  __shared__ double red[RCC];
  if (state[1] == 0.0) return;  // the solve has stopped (uniform; the FVP pass was gated too)
  double* zbuf = work;
  double* pzp = work + P;
  const int t = threadIdx.x, cl = t & (RCC - 1), rl = t / RCC;
  const int c = blockIdx.x * RCC + cl;
  const int nruns = (nb + RB - 1) / RB;  // <= 16: the pass runs at most 256 blocks
  if (c < P && rl < nruns) {
    const int b0 = rl * RB, b1 = min(nb, b0 + RB);
    double sr = 0.0;
#pragma unroll 8
    for (int b = b0; b < b1; ++b) sr += part[(long long)b * P + c];
    runs[rl * RCC + cl] = sr;
  }
  __syncthreads();
  if (rl == 0) {
    double pl = 0.0;
    if (c < P) {
      double h = runs[cl];
      if (nruns > 1) {
        h = 0.0;
        for (int q = 0; q < nruns; ++q) h += runs[q * RCC + cl];  // amx_npg_reduce's second stage
      }
      const double pv = p[c];
      double z = h;
      if (c >= P - A) z += curv[c - (P - A)] * (double)p32[c];
      z += damping * pv;
      zbuf[c] = z;
      pl = pv * z;
    }
    red[cl] = pl;
  }
  __syncthreads();
  if (t == 0) {
    double sp = 0.0;
    for (int q = 0; q < RCC; ++q) sp += red[q];  // the block's columns in order
    pzp[blockIdx.x] = sp;
  }
}

__global__ __launch_bounds__(XRT) void k_npg_cg_xrp(int P, double tol, const double* __restrict__ state_in,
                                                    double* __restrict__ state_out, double* __restrict__ x,
                                                    const double* __restrict__ r_in, double* __restrict__ r_out,
                                                    double* __restrict__ p, float* __restrict__ p32,
                                                    const double* __restrict__ work) {
  __shared__ double red[XRT / 64];
  const int t = threadIdx.x;
  if (state_in[1] == 0.0) {  // stopped: carry r and the state over to the out buffers
    const int e = blockIdx.x * XRT + t;
    if (e < P) r_out[e] = r_in[e];
    if (blockIdx.x == 0 && t == 0) {
      state_out[0] = state_in[0];
      state_out[1] = 0.0;
    }
    return;
  }
  const double* zbuf = work;
  const double rdotr = state_in[0];
  const double v = rdotr / parts_sum(work + P, (P + RCC - 1) / RCC);
  // r'.r' over all P elements in one fixed order (thread t: t, t + XRT, ...; waves in order)
  // (P <= XRT * CGE: the loop unrolled so all its loads are in flight at once, the adds in order)
  double rr = 0.0;
  {
    double rl[CGE], zl[CGE];
#pragma unroll
    for (int u = 0; u < CGE; ++u) {
      const int e = t + u * XRT;
      rl[u] = e < P ? r_in[e] : 0.0;
      zl[u] = e < P ? zbuf[e] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < CGE; ++u) {
      const double rv = rl[u] - v * zl[u];
      rr += rv * rv;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) rr += __shfl_xor(rr, o);
  if ((t & 63) == 0) red[t >> 6] = rr;
  __syncthreads();
  rr = 0.0;
  for (int w = 0; w < XRT / 64; ++w) rr += red[w];
  const double mu = rr / rdotr;
  const int e = blockIdx.x * XRT + t;
  if (e < P) {
    const double pv = p[e];
    x[e] += v * pv;
    const double rv = r_in[e] - v * zbuf[e];
    r_out[e] = rv;
    const double pn = rv + mu * pv;
    p[e] = pn;
    p32[e] = (float)pn;
  }
  if (blockIdx.x == 0 && t == 0) {
    state_out[0] = rr;
    state_out[1] = rr < tol ? 0.0 : 1.0;
  }
}

size_t npg_lds_bytes(int S, int A, int mode, int rc) {
  const Geo g(S, A);
  size_t fl = (size_t)small_floats(g) * (mode == NPG_VPG ? 1 : 2) + r4(rc * g.XS) + 2 * r4(rc * HS) +
              2 * r4(rc * DS) + r4(rc * g.GS) + r4(2 * g.A16);
  if (mode != NPG_FVP) fl += r4(rc * g.GS) + r4(rc * A) + r4(2 * rc);  // M, ACT, ADV
  return fl * sizeof(float);
}

}  // namespace

extern "C" long long amx_npg_param_count(int S, int A) {
  return (long long)NH * S + NH + NH * NH + NH + (long long)A * NH + A + A;
}

extern "C" int amx_npg_pass(amx_ctx* ctx, int mode, int N, const void* obs, int obs_dtype, long long ldo,
                            const void* act, int act_dtype, long long lda, const double* adv, const float* theta,
                            const float* vec, int rows_per_block, double* partials, void* stream) {
  return amx_npg_pass_gated(ctx, mode, N, obs, obs_dtype, ldo, act, act_dtype, lda, adv, theta, vec, rows_per_block,
                            partials, nullptr, stream);
}

extern "C" int amx_npg_pass_gated(amx_ctx* ctx, int mode, int N, const void* obs, int obs_dtype, long long ldo,
                                  const void* act, int act_dtype, long long lda, const double* adv,
                                  const float* theta, const float* vec, int rows_per_block, double* partials,
                                  const double* gate, void* stream) {
  return amx_npg_pass_ex(ctx, mode, N, obs, obs_dtype, ldo, act, act_dtype, lda, adv, theta, vec, rows_per_block,
                         partials, gate, nullptr, stream);
}

namespace {
// the pass launch behind amx_npg_pass_ex / amx_npg_pass_cg (cg: the fold's operands, or null)
int npg_launch(amx_ctx* ctx, int mode, int N, const void* obs, int obs_dtype, long long ldo, const void* act,
               int act_dtype, long long lda, const double* adv, const float* theta, const float* vec,
               int rows_per_block, double* partials, const double* gate, float* hcache, const NpgArgs* cg,
               void* stream) {
  const int S = ctx->S, A = ctx->A;
  NpgArgs a = {};
  if (cg) a = *cg;
  a.mode = mode; a.N = N; a.S = S; a.A = A; a.rows_per_block = rows_per_block;
  a.obs = obs; a.ldo = ldo;
  a.act = act; a.lda = lda;
  a.adv = adv; a.theta = theta; a.vec = vec; a.partials = partials; a.gate = gate; a.hcache = hcache;
  a.P = (int)amx_npg_param_count(S, A);
  const bool of64 = obs_dtype == AMX_IN_F64, af64 = act_dtype == AMX_IN_F64;
  AMX_CHECK_ARG(!hcache || mode == NPG_VPG || (mode == NPG_FVP && !of64),
                "amx_npg_pass: hcache is written by VPG and read by FVP on fp32 observations (mode %d)", mode);
  AMX_CHECK_ARG(((uintptr_t)hcache & 15) == 0, "amx_npg_pass: hcache must be 16-byte aligned");
  const size_t lds = npg_lds_bytes(S, A, mode, RC0);
  AMX_CHECK_ARG(lds <= 160 * 1024, "amx_npg_pass: %zu B of LDS", lds);
  const int blocks = (N + rows_per_block - 1) / rows_per_block;
  // f32 inputs (DeviceNPG casts once per update) get kernels compiled for the layer-1 depth
  // ceil(S / 16) rounded up to 4, 8, 13 or 16 steps; fp64 inputs the 16-step kernel
  const int jj = (S + 15) / 16;
  void (*kern)(NpgArgs) = nullptr;
  if (!of64 && (mode == NPG_FVP || !af64)) {
#define NPG_PICK(J)                                                                                  \
  kern = mode == NPG_FVP ? (hcache ? k_npg<NPG_FVP, float, float, RC0, J, true> : k_npg<NPG_FVP, float, float, RC0, J>) \
       : mode == NPG_VPG ? k_npg<NPG_VPG, float, float, RC0, J> : k_npg<NPG_EVAL, float, float, RC0, J>
    if (jj <= 4) NPG_PICK(4);
    else if (jj <= 8) NPG_PICK(8);
    else if (jj <= 13) NPG_PICK(13);
    else NPG_PICK(16);
#undef NPG_PICK
  } else if (mode == NPG_FVP) {  // actions are not read
    kern = k_npg<NPG_FVP, double, float, RC0, MAXJJ>;
  } else if (mode == NPG_VPG) {
    kern = of64 ? (af64 ? k_npg<NPG_VPG, double, double, RC0, MAXJJ> : k_npg<NPG_VPG, double, float, RC0, MAXJJ>)
                : k_npg<NPG_VPG, float, double, RC0, MAXJJ>;
  } else {
    kern = of64 ? (af64 ? k_npg<NPG_EVAL, double, double, RC0, MAXJJ> : k_npg<NPG_EVAL, double, float, RC0, MAXJJ>)
                : k_npg<NPG_EVAL, float, double, RC0, MAXJJ>;
  }
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(NT), lds, (hipStream_t)stream, a);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}
}  // namespace

extern "C" int amx_npg_pass_ex(amx_ctx* ctx, int mode, int N, const void* obs, int obs_dtype, long long ldo,
                               const void* act, int act_dtype, long long lda, const double* adv, const float* theta,
                               const float* vec, int rows_per_block, double* partials, const double* gate,
                               float* hcache, void* stream) {
  AMX_CHECK_ARG(ctx, "amx_npg_pass: null ctx");
  const int S = ctx->S, A = ctx->A;
  AMX_CHECK_ARG(mode >= NPG_VPG && mode <= NPG_EVAL, "amx_npg_pass: mode=%d", mode);
  AMX_CHECK_ARG(S > 0 && S <= MAXS && A > 0 && A <= MAXA, "amx_npg_pass: S=%d (<= %d), A=%d (<= %d)", S, MAXS, A,
                MAXA);
  AMX_CHECK_ARG(N > 0 && rows_per_block > 0 && rows_per_block % RC0 == 0,
                "amx_npg_pass: N=%d rows_per_block=%d (multiple of %d)", N, rows_per_block, RC0);
  AMX_CHECK_ARG(obs && act && theta && partials, "amx_npg_pass: null buffer");
  AMX_CHECK_ARG((mode == NPG_FVP || adv) && (mode == NPG_VPG || vec), "amx_npg_pass: adv/vec missing for mode %d",
                mode);
  AMX_CHECK_ARG(ldo >= S && lda >= A, "amx_npg_pass: ldo=%lld lda=%lld", ldo, lda);
  AMX_CHECK_ARG(((uintptr_t)theta & 15) == 0 && ((uintptr_t)vec & 15) == 0,
                "amx_npg_pass: theta / vec must be 16-byte aligned (W1 is read as float4s)");
  return npg_launch(ctx, mode, N, obs, obs_dtype, ldo, act, act_dtype, lda, adv, theta, vec, rows_per_block, partials,
                    gate, hcache, nullptr, stream);
}

extern "C" int amx_npg_pass_cg(amx_ctx* ctx, int N, const void* obs, int obs_dtype, long long ldo,
                               const float* theta, int rows_per_block, double* partials, float* hcache, double tol,
                               double* x, const double* r_in, double* r_out, const double* p_in, double* p_out,
                               float* p32_out, const double* state_in, double* state_out, const double* work,
                               void* stream) {
  AMX_CHECK_ARG(ctx, "amx_npg_pass_cg: null ctx");
  const int S = ctx->S, A = ctx->A;
  AMX_CHECK_ARG(S > 0 && S <= MAXS && A > 0 && A <= MAXA, "amx_npg_pass_cg: S=%d (<= %d), A=%d (<= %d)", S, MAXS,
                A, MAXA);
  AMX_CHECK_ARG(N > 0 && rows_per_block > 0 && rows_per_block % RC0 == 0,
                "amx_npg_pass_cg: N=%d rows_per_block=%d (multiple of %d)", N, rows_per_block, RC0);
  AMX_CHECK_ARG(obs && theta && partials && x && r_in && r_out && p_in && p_out && p32_out && state_in && state_out &&
                    work,
                "amx_npg_pass_cg: null buffer");
  AMX_CHECK_ARG(r_in != r_out && p_in != p_out && state_in != state_out,
                "amx_npg_pass_cg: r, p and the state must alternate buffers (every block reads all of them)");
  AMX_CHECK_ARG(ldo >= S && ((uintptr_t)theta & 15) == 0, "amx_npg_pass_cg: ldo=%lld, theta 16-byte aligned", ldo);
  const int P = (int)amx_npg_param_count(S, A);
  const Geo g(S, A);
  // p' (P floats) and the 16 wave sums are staged from the X tile to the end of the LDS image
  const size_t region = npg_lds_bytes(S, A, NPG_FVP, RC0) - sizeof(float) * 2 * small_floats(g);
  AMX_CHECK_ARG(P <= NT * 2 * CGE && sizeof(float) * (r4(P) + 4 * NW) <= region,
                "amx_npg_pass_cg: P=%d does not fit the fold (<= %d, %zu B of staging)", P, NT * 2 * CGE, region);
  NpgArgs cg = {};
  cg.cg_state_in = state_in; cg.cg_state_out = state_out; cg.cg_tol = tol;
  cg.cg_x = x; cg.cg_r_in = r_in; cg.cg_r_out = r_out;
  cg.cg_p_in = p_in; cg.cg_p_out = p_out; cg.cg_p32_out = p32_out; cg.cg_work = work;
  return npg_launch(ctx, NPG_FVP, N, obs, obs_dtype, ldo, obs, AMX_IN_F32, A, nullptr, theta, nullptr,
                    rows_per_block, partials, nullptr, hcache, &cg, stream);
}

extern "C" int amx_npg_reduce(amx_ctx* ctx, const double* partials, int blocks, int P, double* out, void* stream) {
  return amx_npg_reduce_gated(ctx, partials, blocks, P, out, nullptr, stream);
}

extern "C" int amx_npg_reduce_gated(amx_ctx* ctx, const double* partials, int blocks, int P, double* out,
                                    const double* gate, void* stream) {
  AMX_CHECK_ARG(ctx && partials && out && blocks > 0 && P > 0, "amx_npg_reduce: bad arguments");
  const int runs = (blocks + RB - 1) / RB;
  if (runs == 1) {
    hipLaunchKernelGGL(k_npg_reduce2, dim3((P + 255) / 256), dim3(256), 0, (hipStream_t)stream, partials, blocks, P,
                       out, gate);
    AMX_CHECK_LAUNCH();
    return AMX_OK;
  }
  // the runs' sums go to a context-owned scratch (grown on demand, freed with the context)
  const size_t need = sizeof(double) * (size_t)runs * P;
  if (ctx->npg_scratch_bytes < need) {
    if (ctx->d_npg_scratch) AMX_CHECK_HIP(hipFree(ctx->d_npg_scratch));
    ctx->d_npg_scratch = nullptr;
    ctx->npg_scratch_bytes = 0;
    if (hipMalloc((void**)&ctx->d_npg_scratch, need) != hipSuccess) {
      amx::set_error("amx_npg_reduce: hipMalloc of %zu B failed", need);
      return AMX_E_NOMEM;
    }
    ctx->npg_scratch_bytes = need;
  }
  hipLaunchKernelGGL(k_npg_reduce1, dim3((P + 255) / 256, runs), dim3(256), 0, (hipStream_t)stream, partials, blocks,
                     P, ctx->d_npg_scratch, gate);
  AMX_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_npg_reduce2, dim3((P + 255) / 256), dim3(256), 0, (hipStream_t)stream, ctx->d_npg_scratch,
                     runs, P, out, gate);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" long long amx_npg_cg_tail_work(int P) { return (long long)P + (P + RCC - 1) / RCC; }

extern "C" int amx_npg_cg_tail(amx_ctx* ctx, const double* partials, int blocks, int P, int A, const double* curv,
                               double damping, double tol, double* x, const double* r_in, double* r_out, double* p,
                               float* p32, const double* state_in, double* state_out, double* work, void* stream) {
  AMX_CHECK_ARG(ctx && partials && curv && x && r_in && r_out && p && p32 && state_in && state_out && work,
                "amx_npg_cg_tail: null argument");
  AMX_CHECK_ARG(r_in != r_out && state_in != state_out, "amx_npg_cg_tail: r and the state must alternate buffers");
  AMX_CHECK_ARG(blocks > 0 && blocks <= RB * RCT / RCC && P > A && A > 0 && P <= XRT * CGE,
                "amx_npg_cg_tail: blocks=%d (<= %d) P=%d A=%d (P <= %d)", blocks, RB * RCT / RCC, P, A, XRT * CGE);
  const hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_npg_cg_reduce, dim3((P + RCC - 1) / RCC), dim3(RCT), 0, s, partials, blocks, P, A, curv,
                     damping, p, p32, state_in, work);
  AMX_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_npg_cg_xrp, dim3((P + XRT - 1) / XRT), dim3(XRT), 0, s, P, tol, state_in, state_out, x, r_in,
                     r_out, p, p32, work);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_npg_cg_reduce(amx_ctx* ctx, const double* partials, int blocks, int P, int A, const double* curv,
                                 double damping, const double* p, const float* p32, const double* state, double* work,
                                 void* stream) {
  AMX_CHECK_ARG(ctx && partials && curv && p && p32 && state && work, "amx_npg_cg_reduce: null argument");
  AMX_CHECK_ARG(blocks > 0 && blocks <= RB * RCT / RCC && P > A && A > 0 && P <= XRT * CGE,
                "amx_npg_cg_reduce: blocks=%d (<= %d) P=%d A=%d (P <= %d)", blocks, RB * RCT / RCC, P, A, XRT * CGE);
  hipLaunchKernelGGL(k_npg_cg_reduce, dim3((P + RCC - 1) / RCC), dim3(RCT), 0, (hipStream_t)stream, partials, blocks,
                     P, A, curv, damping, p, p32, state, work);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_npg_cg_xrp(amx_ctx* ctx, int P, double tol, double* x, const double* r_in, double* r_out,
                              double* p, float* p32, const double* state_in, double* state_out, const double* work,
                              void* stream) {
  AMX_CHECK_ARG(ctx && x && r_in && r_out && p && p32 && state_in && state_out && work,
                "amx_npg_cg_xrp: null argument");
  AMX_CHECK_ARG(r_in != r_out && state_in != state_out, "amx_npg_cg_xrp: r and the state must alternate buffers");
  AMX_CHECK_ARG(P > 0 && P <= XRT * CGE, "amx_npg_cg_xrp: P=%d (<= %d)", P, XRT * CGE);
  hipLaunchKernelGGL(k_npg_cg_xrp, dim3((P + XRT - 1) / XRT), dim3(XRT), 0, (hipStream_t)stream, P, tol, state_in,
                     state_out, x, r_in, r_out, p, p32, work);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_npg_curvature(amx_ctx* ctx, const float* theta, int P, int A, double* curv, void* stream) {
  AMX_CHECK_ARG(ctx && theta && curv && P > A && A > 0, "amx_npg_curvature: bad arguments");
  hipLaunchKernelGGL(k_npg_curvature, dim3((A + 63) / 64), dim3(64), 0, (hipStream_t)stream, theta, P, A, curv);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_npg_apply_step(amx_ctx* ctx, int P, int A, const double* vpg, const double* npg,
                                  const float* theta, int use_alpha, double alpha, double n_step_size,
                                  float min_log_std, float* new_theta, double* scal, void* stream) {
  AMX_CHECK_ARG(ctx && vpg && npg && theta && new_theta && scal, "amx_npg_apply_step: null argument");
  AMX_CHECK_ARG(P > A && A > 0 && P <= CGT * CGE, "amx_npg_apply_step: P=%d A=%d (P <= %d)", P, A, CGT * CGE);
  hipLaunchKernelGGL(k_npg_apply, dim3(1), dim3(CGT), 0, (hipStream_t)stream, P, A, vpg, npg, theta, use_alpha, alpha,
                     n_step_size, min_log_std, new_theta, scal);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_npg_cg_init(amx_ctx* ctx, int P, const double* b, double* x, double* r, double* p, float* p32,
                               double* state, void* stream) {
  AMX_CHECK_ARG(ctx && b && x && r && p && p32 && state, "amx_npg_cg_init: null argument");
  AMX_CHECK_ARG(P > 0 && P <= CGT * CGE, "amx_npg_cg_init: P=%d (<= %d)", P, CGT * CGE);
  hipLaunchKernelGGL(k_npg_cg_init, dim3(1), dim3(CGT), 0, (hipStream_t)stream, P, b, x, r, p, p32, state, 0,
                     nullptr, nullptr);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_npg_cg_init_ls(amx_ctx* ctx, int P, int A, const float* theta, double* curv, const double* b,
                                  double* x, double* r, double* p, float* p32, double* state, void* stream) {
  AMX_CHECK_ARG(ctx && theta && curv && b && x && r && p && p32 && state, "amx_npg_cg_init_ls: null argument");
  AMX_CHECK_ARG(P > 0 && P <= CGT * CGE && A > 0 && A < P, "amx_npg_cg_init_ls: P=%d A=%d (P <= %d)", P, A,
                CGT * CGE);
  hipLaunchKernelGGL(k_npg_cg_init, dim3(1), dim3(CGT), 0, (hipStream_t)stream, P, b, x, r, p, p32, state, A, theta,
                     curv);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

extern "C" int amx_npg_cg_step(amx_ctx* ctx, int P, int A, const double* h, const double* curv, double damping,
                               double residual_tol, double* x, double* r, double* p, float* p32, double* state,
                               void* stream) {
  AMX_CHECK_ARG(ctx && h && curv && x && r && p && p32 && state, "amx_npg_cg_step: null argument");
  AMX_CHECK_ARG(P > 0 && P <= CGT * CGE && A > 0 && A <= P, "amx_npg_cg_step: P=%d A=%d", P, A);
  hipLaunchKernelGGL(k_npg_cg_step, dim3(1), dim3(CGT), 0, (hipStream_t)stream, P, A, h, curv, damping,
                     residual_tol, x, r, p, p32, state);
  AMX_CHECK_LAUNCH();
  return AMX_OK;
}

#ifdef NPG_TRACE
extern "C" int amx_npg_trace_read(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(npg_trace_buf), sizeof(unsigned long long) * 4 * 64) == hipSuccess ? 0 : 1;
}
#endif
