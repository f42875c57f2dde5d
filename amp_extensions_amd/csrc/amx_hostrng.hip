// Host-side policy noise of the reference's sampler, bit-exact: numpy's legacy RandomState
// stream (MT19937 seeded by np.random.seed(int), mt19937_seed / mt19937_gen / legacy_double /
// legacy_gauss of numpy's random module) as mjrl's MLP.get_action consumes it
// (mjrl/mjrl/policies/gaussian_mlp.py:95-104): per step one np.random.uniform() for the eps
// test, then np.random.randn(A) -- with the polar method's cached second normal carried across
// calls.  Trajectory j of sampler worker i is seeded with 12345 + base_seed * i + j
// (milo/milo/sampler.py:33-40, 116-121).
//
// sample_points (amp_extensions_amd/sampler.py) keeps one generator state per lane and draws
// each chunk's noise for the lanes in flight with one call, instead of ~2 numpy calls per lane
// and step.  Plain C++ on the host (no device code); lanes are split over threads.  The libm
// log/sqrt are the ones numpy's legacy_gauss calls, and -ffp-contract=off keeps the
// x1*x1 + x2*x2 rounding of numpy's baseline-x86-64 build.
#include <math.h>
#include <stdint.h>

#include <thread>
#include <vector>

#include "amx_common.h"

namespace {

constexpr int kN = 624, kM = 397;

struct MtState {
  uint32_t key[kN];
  int32_t pos;
  int32_t has_gauss;
  double gauss;
};
static_assert(sizeof(MtState) == AMX_MT_STATE_BYTES, "AMX_MT_STATE_BYTES out of date");

void mt_seed(MtState* s, uint32_t seed) {
  for (int p = 0; p < kN; ++p) {
    s->key[p] = seed;
    seed = 1812433253u * (seed ^ (seed >> 30)) + (uint32_t)(p + 1);
  }
  s->pos = kN;
  s->has_gauss = 0;
  s->gauss = 0.0;
}

void mt_gen(MtState* s) {
  constexpr uint32_t upper = 0x80000000u, lower = 0x7fffffffu, matrix = 0x9908b0dfu;
  uint32_t y;
  int i = 0;
  for (; i < kN - kM; ++i) {
    y = (s->key[i] & upper) | (s->key[i + 1] & lower);
    s->key[i] = s->key[i + kM] ^ (y >> 1) ^ (-(y & 1u) & matrix);
  }
  for (; i < kN - 1; ++i) {
    y = (s->key[i] & upper) | (s->key[i + 1] & lower);
    s->key[i] = s->key[i + (kM - kN)] ^ (y >> 1) ^ (-(y & 1u) & matrix);
  }
  y = (s->key[kN - 1] & upper) | (s->key[0] & lower);
  s->key[kN - 1] = s->key[kM - 1] ^ (y >> 1) ^ (-(y & 1u) & matrix);
  s->pos = 0;
}

inline uint32_t mt_next(MtState* s) {
  if (s->pos == kN) mt_gen(s);
  uint32_t y = s->key[s->pos++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

inline double mt_double(MtState* s) {  // 53-bit uniform in [0, 1)
  const int32_t a = (int32_t)(mt_next(s) >> 5), b = (int32_t)(mt_next(s) >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}

inline double mt_gauss(MtState* s) {  // legacy polar Box-Muller with the cached second value
  if (s->has_gauss) {
    const double g = s->gauss;
    s->has_gauss = 0;
    s->gauss = 0.0;
    return g;
  }
  double x1, x2, r2;
  do {
    x1 = 2.0 * mt_double(s) - 1.0;
    x2 = 2.0 * mt_double(s) - 1.0;
    r2 = x1 * x1 + x2 * x2;
  } while (r2 >= 1.0 || r2 == 0.0);
  const double f = sqrt(-2.0 * log(r2) / r2);
  s->gauss = f * x1;
  s->has_gauss = 1;
  return f * x2;
}

template <class F>
void parallel_for(int n, F&& body) {
  const unsigned hw = std::thread::hardware_concurrency();
  const int nt = (int)std::min<unsigned>(hw ? hw : 1u, 16u);
  if (n < 32 || nt <= 1) {
    for (int i = 0; i < n; ++i) body(i);
    return;
  }
  std::vector<std::thread> th;
  const int per = (n + nt - 1) / nt;
  for (int t = 0; t < nt; ++t) {
    const int lo = t * per, hi = std::min(n, lo + per);
    if (lo >= hi) break;
    th.emplace_back([lo, hi, &body] {
      for (int i = lo; i < hi; ++i) body(i);
    });
  }
  for (auto& x : th) x.join();
}

}  // namespace

extern "C" int amx_mt_seed(void* states, int n_states, const int32_t* slots, const uint32_t* seeds, int n) {
  AMX_CHECK_ARG(states && slots && seeds && n >= 0 && n_states >= 0, "amx_mt_seed: bad arguments");
  for (int i = 0; i < n; ++i)
    AMX_CHECK_ARG(slots[i] >= 0 && slots[i] < n_states, "amx_mt_seed: slot %d of %d", slots[i], n_states);
  MtState* st = (MtState*)states;
  for (int i = 0; i < n; ++i) mt_seed(st + slots[i], seeds[i]);
  return AMX_OK;
}

extern "C" int amx_mt_policy_noise(void* states, int n_states, const int32_t* slots, int n, int steps, int A,
                                   double* out, long long ld_step, long long ld_slot) {
  AMX_CHECK_ARG(states && slots && out && n >= 0 && steps >= 0 && A > 0, "amx_mt_policy_noise: bad arguments");
  for (int i = 0; i < n; ++i)
    AMX_CHECK_ARG(slots[i] >= 0 && slots[i] < n_states, "amx_mt_policy_noise: slot %d of %d", slots[i], n_states);
  MtState* st = (MtState*)states;
  parallel_for(n, [&](int i) {
    MtState* s = st + slots[i];
    double* o = out + (long long)slots[i] * ld_slot;
    for (int k = 0; k < steps; ++k) {
      (void)mt_double(s);  // np.random.uniform() < eps (gaussian_mlp.py:99)
      for (int a = 0; a < A; ++a) o[(long long)k * ld_step + a] = mt_gauss(s);  // np.random.randn(A)
    }
  });
  return AMX_OK;
}
