// Shared definitions of the split16 kernels (edge16.hip: the edge GEMMs on 16x16x32 MFMA, split16.hip:
// operand preparation). Included inside namespace chm.
#pragma once

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

namespace {

constexpr int BM = 256, BN = 256, BK = 32;
constexpr int NSA = 3, NSW = 2;             // ring depths: A (streamed from HBM) and W (L2-resident)
constexpr int ROW_B = BK * 2 * 2;           // one row of a K-tile: 32 hi + 32 lo fp16 = one 128-B line
constexpr int OPND_B = BM * ROW_B;          // 32 KB per operand tile
constexpr int W_RING = NSA * OPND_B;        // W stages follow the A stages
constexpr int RING_B = (NSA + NSW) * OPND_B;  // 160 KB
constexpr int SEG_TP = 132;                 // EPI_SEGMEAN column tile pitch (floats)
constexpr int SEG_B = BM * SEG_TP * 4;      // 135168 B
constexpr int LDS_B = RING_B > SEG_B + 2048 ? RING_B : SEG_B + 2048;  // (+ the SEGMEAN node list)
constexpr int CHUNK = 128;                  // S scale granularity (columns)
constexpr int PQ_PITCH = 260;               // EPI_EDGE staged P / Q rows (floats)
constexpr int PQ_OFF = 0;
// P / Q rows staged by the main loop's last iterations (EPI_EDGE, K = 768): conditioning 0 at row 0
// (A stages 0-1, free after the barrier of K-tile nk-2), conditioning 1 at row PRE_ROW1 (free after
// the barrier of nk-1); both images hold up to PRE_MAX rows
constexpr int PRE_ROW1 = 63, PRE_MAX = 61;

__device__ __forceinline__ float silu_e(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.44269504088896341f * x));
}
// the same on a pair, written with 2-wide vectors so the multiplies and adds issue packed
// (v_pk_mul_f32 / v_pk_add_f32: half the VALU slots; bit-identical to silu_e per element)
typedef float f32x2e __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2e silu_e2(f32x2e x) {
  f32x2e t = x * -1.44269504088896341f;
  t.x = __builtin_amdgcn_exp2f(t.x);
  t.y = __builtin_amdgcn_exp2f(t.y);
  t = t + 1.0f;
  t.x = __builtin_amdgcn_rcpf(t.x);
  t.y = __builtin_amdgcn_rcpf(t.y);
  return x * t;
}

__device__ __forceinline__ long remap(long b, long nb) {
  const long q = nb / 8, r = nb % 8, xcd = b % 8, idx = b / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

__device__ __forceinline__ unsigned long long rtime() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}
__device__ __forceinline__ unsigned long long ctime() {  // shader clock counter
  unsigned long long t;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}
__device__ __forceinline__ unsigned hwid() {
  unsigned hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  return ((xcc & 0xf) << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xf);
}

// exponent e with m = f 2^e, f in [0.5, 1) (0 for m == 0)
__device__ __forceinline__ int exp_of(float m) {
  int e = 0;
  if (m > 0.f) frexpf(m, &e);
  return e;
}

}  // namespace
