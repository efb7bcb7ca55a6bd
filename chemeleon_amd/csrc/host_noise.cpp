// Host side of parity-mode noise: the uniform draws of the reference's CPU RNG stream.
//
// The reference samples its atom-type noise as torch.rand(N, A) on the CPU generator every reverse
// step (chemeleon/modules/chemeleon.py:400-404). torch's CPU generator is an MT19937 engine
// (ATen's mt19937_engine) and a float uniform takes one 32-bit output y per element, kept as
// (y & (2^24 - 1)) * 2^-24 (at::uniform_real_distribution<float> on CPUGeneratorImpl::random()).
// A rank of a sample-parallel run needs only its own rows of that tensor, but the stream is
// sequential: every rank advances the engine over the whole global tensor. This routine does that
// without tempering or converting the outputs it does not keep: 1.1 ms for the 64x40 rows of the
// 512x40 tensor against 9.2 ms for torch.rand of the whole tensor (one core of the CPU container), so
// the draw hides under the per-GPU reverse step.
#include <cstdint>
#include <cstring>

#include "../../include/chemeleon_hip.h"

int chm_fail_host(int code, const char* msg);  // runtime.hip: sets chm_last_error()

namespace {
constexpr int kN = 624, kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;

inline uint32_t twist(uint32_t u, uint32_t v) {
  return (((u & kUpper) | (v & kLower)) >> 1) ^ ((v & 1u) ? kMatrixA : 0u);
}

// ATen's mt19937_engine::next_state
void next_state(uint32_t* s) {
  int i = 0;
  for (; i < kN - kM; ++i) s[i] = s[i + kM] ^ twist(s[i], s[i + 1]);
  for (; i < kN - 1; ++i) s[i] = s[i + kM - kN] ^ twist(s[i], s[i + 1]);
  s[kN - 1] = s[kM - 1] ^ twist(s[kN - 1], s[0]);
}

inline float temper_uniform(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return (float)(y & 0xffffffu) * (1.0f / 16777216.0f);  // exact: a 24-bit integer times 2^-24
}
}  // namespace

extern "C" int chm_mt19937_uniform(uint32_t* state, int32_t* left, int32_t* next, int64_t count, int64_t lo,
                                   int64_t hi, float* out) {
  if (!state || !left || !next || count < 0 || lo < 0 || hi < lo || hi > count || (hi > lo && !out))
    return chm_fail_host(CHM_E_ARG, "chm_mt19937_uniform: NULL pointer or [lo, hi) outside [0, count)");
  if (*left < 1 || *left > kN || *next < 0 || *next > kN || (*left > 1 && *next + *left != kN + 1))
    return chm_fail_host(CHM_E_ARG, "chm_mt19937_uniform: engine position outside the MT19937 state");
  int l = *left, nx = *next;
  int64_t i = 0;
  while (i < count) {
    // torch: `if (--left == 0) next_state();` before each output, so the engine twists when left is 1
    if (l == 1) {
      next_state(state);
      l = kN + 1;
      nx = 0;
    }
    // outputs available before the next twist: l - 1
    int64_t run = l - 1;
    if (run > count - i) run = count - i;
    int64_t a = i > lo ? i : lo, b = (i + run) < hi ? (i + run) : hi;
    for (int64_t k = a; k < b; ++k) out[k - lo] = temper_uniform(state[nx + (k - i)]);
    nx += (int)run;
    l -= (int)run;
    i += run;
  }
  *left = l;
  *next = nx;
  return CHM_OK;
}
