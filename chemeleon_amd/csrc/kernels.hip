// Device kernels of the Chemeleon sampling path for MI355X (gfx950, CDNA4).
//
// Numerics: every product / sum is fp32 (v_mfma_f32_32x32x2_f32 is an exact
// fp32 fma chain); the elementwise step updates use explicitly rounded
// __fmul_rn / __fadd_rn so hipcc cannot contract them into FMAs that the
// reference's separate ATen ops do not perform.
#include "chm_internal.h"

#include <math.h>

namespace chm {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float silu(float x) { return x / (1.0f + expf(-x)); }

// torch.remainder(x, 1.0) for fp32: fmod, then shift negatives by +1
// (can return exactly 1.0 for tiny negatives, as the reference does).
__device__ __forceinline__ float rem1(float x) {
  float m = fmodf(x, 1.0f);
  if (m != 0.0f && m < 0.0f) m = __fadd_rn(m, 1.0f);
  return m;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// A 512-column row held by one wave as 2 x float4 per lane (columns 4 lane .. +3 and 256 + 4 lane .. +3)
// written as a split row for the pre-split node GEMMs (GemmArgs::aex): [H/16][hi 16 | lo 16] fp16 of the
// row scaled by 2^-e per 128-column chunk (chunk = lanes 0-31 / 32-63 of v0, then of v1), e the exponent of
// the chunk's max |value|; ex[row] = the 4 exponents as packed int8.
typedef _Float16 f16x4k __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int exp_of_k(float m) {
  int e = 0;
  if (m > 0.f) frexpf(m, &e);
  return e;
}
__device__ __forceinline__ void store_split_row512(const f32x4& v0, const f32x4& v1, int lane, void* rows, int* ex,
                                                   long r) {
  float m0 = fmaxf(fmaxf(fabsf(v0.x), fabsf(v0.y)), fmaxf(fabsf(v0.z), fabsf(v0.w)));
  float m1 = fmaxf(fmaxf(fabsf(v1.x), fabsf(v1.y)), fmaxf(fabsf(v1.z), fabsf(v1.w)));
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) {  // within each half-wave: one 128-column chunk
    m0 = fmaxf(m0, __shfl_xor(m0, o, 64));
    m1 = fmaxf(m1, __shfl_xor(m1, o, 64));
  }
  const int e0 = exp_of_k(m0), e1 = exp_of_k(m1);
  _Float16* out = reinterpret_cast<_Float16*>(rows) + r * (2L * H);
  const f32x4 vv[2] = {v0, v1};
  const int ee[2] = {e0, e1};
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const float sc = ldexpf(1.0f, -ee[p]);
    const int col = 256 * p + 4 * lane;
    f16x4k hi, lo;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float x = vv[p][k] * sc;
      hi[k] = (_Float16)x;
      lo[k] = (_Float16)(x - (float)hi[k]);
    }
    *reinterpret_cast<f16x4k*>(out + (col >> 4) * 32 + (col & 15)) = hi;
    *reinterpret_cast<f16x4k*>(out + (col >> 4) * 32 + 16 + (col & 15)) = lo;
  }
  const int e0b = __shfl(e0, 32, 64), e1b = __shfl(e1, 32, 64);
  if (lane == 0) ex[r] = (e0 & 255) | ((e0b & 255) << 8) | ((e1 & 255) << 16) | ((e1b & 255) << 24);
}

// ---------------------------------------------------------------------------
// Philox4x32-10 (counter-based): perf-mode noise keyed by (seed, t, index)
// ---------------------------------------------------------------------------
struct U4 { uint32_t x, y, z, w; };
__device__ __forceinline__ U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
    uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
    uint32_t n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
    c0 = n0; c1 = l1; c2 = n2; c3 = l0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return U4{c0, c1, c2, c3};
}
// kind: 0 atom-type uniforms, 1 lattice normals, 2 / 3 coordinate normals
__device__ __forceinline__ float rng_uniform(uint64_t seed, int t, int kind, uint64_t idx) {
  U4 r = philox((uint32_t)idx, (uint32_t)(idx >> 32), (uint32_t)t, (uint32_t)kind, (uint32_t)seed,
                (uint32_t)(seed >> 32));
  return (float)(r.x >> 8) * (1.0f / 16777216.0f);  // [0, 1)
}
__device__ __forceinline__ float rng_normal(uint64_t seed, int t, int kind, uint64_t idx) {
  U4 r = philox((uint32_t)idx, (uint32_t)(idx >> 32), (uint32_t)t, (uint32_t)kind | 0x100u, (uint32_t)seed,
                (uint32_t)(seed >> 32));
  float u1 = ((float)(r.x >> 8) + 1.0f) * (1.0f / 16777216.0f);  // (0, 1]
  float u2 = (float)(r.y >> 8) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
}

// the perf-mode streams themselves, for their statistical tests (chm_debug_philox)
__global__ void k_philox_fill(uint64_t seed, int t, int kind, int64_t base, long n, int normal, float* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = normal ? rng_normal(seed, t, kind, (uint64_t)(base + i)) : rng_uniform(seed, t, kind, (uint64_t)(base + i));
}
hipError_t philox_fill(uint64_t seed, int t, int kind, int64_t base, long n, int normal, float* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_philox_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, seed, t, kind, base, n, normal,
                     out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// GEMM  C = epi(A . W^T) on fp32 MFMA. 128x128x16 tiles, 4 waves in 2x2, each
// wave 64x64 = 2x2 v_mfma_f32_32x32x2_f32 accumulators. Within a 16-deep K
// chunk, k-step s of lane half h reads k = 8h + s, so each lane fetches its
// eight A and eight W values with two ds_read_b128. LDS rows padded to 20
// floats. Register double buffering of the next chunk's global loads.
// ---------------------------------------------------------------------------
constexpr int BM = 128, BN = 128, BK = 16, LDP = 20;

template <int EPI>
__global__ __launch_bounds__(256) void k_gemm(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) float As[2][BM * LDP];
  __shared__ __attribute__((aligned(16))) float Ws[2][BN * LDP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int ntn = g.N / BN;
  const long bm = blockIdx.x / ntn;
  const int bn = blockIdx.x % ntn;
  const long m0 = bm * BM;
  const int n0 = bn * BN;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  f32x4 ra[2], rw[2];
  auto gload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = tid + 256 * q;
      const int row = idx >> 2, c4 = idx & 3;
      const long m = m0 + row;
      const int k = k0 + 4 * c4;
      if (m < g.M) {
        const float* src = (k < g.ksplit) ? g.A + m * g.lda + k : g.A2 + m * g.lda2 + (k - g.ksplit);
        ra[q] = *reinterpret_cast<const f32x4*>(src);
      } else {
        ra[q] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      rw[q] = *reinterpret_cast<const f32x4*>(g.W + (long)(n0 + row) * g.ldw + k);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = tid + 256 * q;
      const int row = idx >> 2, c4 = idx & 3;
      *reinterpret_cast<f32x4*>(&As[buf][row * LDP + 4 * c4]) = ra[q];
      *reinterpret_cast<f32x4*>(&Ws[buf][row * LDP + 4 * c4]) = rw[q];
    }
  };

  const int h = lane >> 5, r32 = lane & 31;
  const int nk = g.K / BK;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);
    f32x4 av[2][2], bv[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float* pa = &As[buf][(wm * 64 + i * 32 + r32) * LDP + 8 * h];
      av[i][0] = *reinterpret_cast<const f32x4*>(pa);
      av[i][1] = *reinterpret_cast<const f32x4*>(pa + 4);
      const float* pw = &Ws[buf][(wn * 64 + i * 32 + r32) * LDP + 8 * h];
      bv[i][0] = *reinterpret_cast<const f32x4*>(pw);
      bv[i][1] = *reinterpret_cast<const f32x4*>(pw + 4);
    }
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][s >> 2][s & 3], bv[j][s >> 2][s & 3], acc[i][j], 0, 0, 0);
    if (kt + 1 < nk) {
      lstore(buf ^ 1);
    }
    __syncthreads();
  }

  // epilogue: acc[i][j][r] -> row (r&3) + 8(r>>2) + 4h, col r32 of the 32x32 tile
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (row >= g.M) continue;
      if (EPI == EPI_EDGE) {
        const long ii = g.ei[row], jj = g.ej[row];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int col = n0 + wn * 64 + j * 32 + r32;
          const float v = acc[i][j][r];
          for (int c = 0; c < g.npairs; ++c) {
            const float p = g.PQ[(c * g.nnodes + ii) * (2 * H) + col];
            const float q = g.PQ[(c * g.nnodes + jj) * (2 * H) + H + col];
            g.C[((long)c * g.E + row) * g.ldc + col] = silu((v + p) + q);
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int col = n0 + wn * 64 + j * 32 + r32;
          float v = acc[i][j][r];
          if (g.bias) v += g.bias[col];
          if (g.gb && col < g.gb_cols) v += g.gb[(long)g.row2g[row % g.gb_rowmod] * g.ldgb + col];
          if (g.act == 1) v = silu(v);
          if (g.R) v += g.R[row * g.ldr + col];
          g.C[row * g.ldc + col] = v;
        }
      }
    }
  }
}

hipError_t gemm(const GemmArgs& g, int epi, hipStream_t s) {
  if (g.N % BN || g.K % BK || g.M <= 0) return hipErrorInvalidValue;
  if (epi == EPI_STD && g.ksplit % BK) return hipErrorInvalidValue;
  const long blocks = ((g.M + BM - 1) / BM) * (g.N / BN);
  if (epi == EPI_EDGE)
    hipLaunchKernelGGL(k_gemm<EPI_EDGE>, dim3((unsigned)blocks), dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL(k_gemm<EPI_STD>, dim3((unsigned)blocks), dim3(256), 0, s, g);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Fourier edge features (cspnet.py:38-52,324): F[e] = [sin(d (x) f) | cos(d (x) f)],
// d = (x_j - x_i) mod 1, f_k = fl32(fl32(2 pi) * k), axis-major within each half.
// ---------------------------------------------------------------------------
__global__ void k_fourier(const float* __restrict__ x, const int* __restrict__ ei, const int* __restrict__ ej, long E,
                          float* __restrict__ F) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= E * 3 * NF) return;
  const long e = idx / (3 * NF);
  const int r = (int)(idx - e * 3 * NF);
  const int a = r / NF, k = r - a * NF;
  const float d = rem1(__fsub_rn(x[(long)ej[e] * 3 + a], x[(long)ei[e] * 3 + a]));
  const float f = __fmul_rn(6.28318548202514648f, (float)k);
  const float arg = __fmul_rn(d, f);
  F[e * FD + r] = sinf(arg);
  F[e * FD + 3 * NF + r] = cosf(arg);
}

hipError_t fourier(const float* x, const int* ei, const int* ej, long E, float* F, hipStream_t s) {
  const long n = E * 3 * NF;
  hipLaunchKernelGGL(k_fourier, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, ei, ej, E, F);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Message-passing aggregation (scatter.py:88-112): agg[c][i] = sum_j msg[c][e0(i)+j] / n_g.
// One 128-thread block per (c, i), one float4 column group per thread,
// rows summed in edge order j = 0..n-1 like the reference's scatter_add_.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(128) void k_segment_mean(const float* __restrict__ msg, float* __restrict__ agg,
                                                      const int* __restrict__ n2g, const int* __restrict__ node_off,
                                                      const long* __restrict__ edge_off, const int* __restrict__ natoms,
                                                      long N, long E) {
  const long b = blockIdx.x;
  const long c = b / N, i = b - c * N;
  const int gph = n2g[i];
  const int n = natoms[gph];
  const long e0 = edge_off[gph] + (i - node_off[gph]) * (long)n;
  const f32x4* src = reinterpret_cast<const f32x4*>(msg + (c * E + e0) * H) + threadIdx.x;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  int j = 0;
  for (; j + 4 <= n; j += 4) {
    f32x4 v0 = src[(long)(j + 0) * (H / 4)];
    f32x4 v1 = src[(long)(j + 1) * (H / 4)];
    f32x4 v2 = src[(long)(j + 2) * (H / 4)];
    f32x4 v3 = src[(long)(j + 3) * (H / 4)];
    s += v0; s += v1; s += v2; s += v3;
  }
  for (; j < n; ++j) s += src[(long)j * (H / 4)];
  const float cnt = n < 1 ? 1.0f : (float)n;
  f32x4 o = {s.x / cnt, s.y / cnt, s.z / cnt, s.w / cnt};
  reinterpret_cast<f32x4*>(agg + b * H)[threadIdx.x] = o;
}

hipError_t segment_mean(const float* msg, float* agg, const int* n2g, const int* node_off, const long* edge_off,
                        const int* natoms, long N, long E, int P, hipStream_t s) {
  hipLaunchKernelGGL(k_segment_mean, dim3((unsigned)(N * P)), dim3(H / 4), 0, s, msg, agg, n2g, node_off, edge_off,
                     natoms, N, E);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// small node / graph kernels
// ---------------------------------------------------------------------------
// per-graph part of edge layer 1 for up to kGBLayers layers: out[l][g][n] = b1_l[n] + sum_ab W1_l[n, ab] (L L^T)_ab
// (cspnet.py:144-152, the C block of W1); element idx = g * H + n of layer l
__device__ __forceinline__ void graph_bias_elem(long idx, int l, const float* __restrict__ lat, const GraphBiasArgs& a,
                                                long ldwc, float* __restrict__ out, int B) {
  const float* Wc = a.Wc[l];
  const int gph = (int)(idx / H), n = (int)(idx % H);
  const float* L = lat + gph * 9;
  float v = a.b1[l][n];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float ip = L[i * 3 + 0] * L[j * 3 + 0] + L[i * 3 + 1] * L[j * 3 + 1] + L[i * 3 + 2] * L[j * 3 + 2];
      v += Wc[n * ldwc + i * 3 + j] * ip;
    }
  out[(long)l * B * H + idx] = v;
}

// one wave per row (4 rows per block); rmax != null: the row's max |value| for the split16 node GEMMs.
// Blocks past the embedding rows (nbe of them) compute the per-graph terms of the first nl layers (nbg blocks
// each; graph_bias' work, folded into this launch: one launch less per decoder call)
__global__ __launch_bounds__(256) void k_embed(const int64_t* __restrict__ a, const float* __restrict__ emb,
                                               float* __restrict__ Hout, long N, int P, float* __restrict__ rmax,
                                               void* Hs, int* He, long nbe, const float* __restrict__ lat,
                                               GraphBiasArgs ga, long ldwc, float* __restrict__ gout, int B, long nbg,
                                               long nbgt, unsigned* __restrict__ z0, long n0, unsigned* __restrict__ z1,
                                               long n1) {
  if ((long)blockIdx.x >= nbe + nbgt) {  // the call's cleared words (the pair grid's repair requests and flags)
    const long idx = ((long)blockIdx.x - nbe - nbgt) * 256 + threadIdx.x;
    if (idx < n0) z0[idx] = 0u;
    else if (idx - n0 < n1) z1[idx - n0] = 0u;
    return;
  }
  if ((long)blockIdx.x >= nbe) {
    const long gb = (long)blockIdx.x - nbe;
    const long idx = (gb % nbg) * 256 + threadIdx.x;
    if (idx < (long)B * H) graph_bias_elem(idx, (int)(gb / nbg), lat, ga, ldwc, gout, B);
    return;
  }
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= N * P) return;
  const f32x4* e4 = reinterpret_cast<const f32x4*>(emb + a[r % N] * H);
  const f32x4 v0 = e4[lane], v1 = e4[64 + lane];
  f32x4* h4 = reinterpret_cast<f32x4*>(Hout + r * H);
  h4[lane] = v0;
  h4[64 + lane] = v1;
  if (rmax) {
    float m = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) m = fmaxf(m, fmaxf(fabsf(v0[k]), fabsf(v1[k])));
    m = wave_max(m);
    if (lane == 0) rmax[r] = m;
  }
  if (Hs) store_split_row512(v0, v1, lane, Hs, He, r);
}
hipError_t embed(const int64_t* a, const float* emb, float* Hout, long N, int P, hipStream_t s, float* rmax, void* Hs,
                 int* He, const float* lat, const GraphBiasArgs* ga, int nl, long ldwc, float* gout, int B, unsigned* z0,
                 long n0, unsigned* z1, long n1) {
  const long rows = N * P;
  const long nbe = (rows + 3) / 4;
  const long nbg = ga ? ((long)B * H + 255) / 256 : 0, nbgt = ga ? nbg * nl : 0;
  if (ga && (nl < 1 || nl > kGBLayers || !lat || !gout || B < 1)) return hipErrorInvalidValue;
  if (n0 < 0 || n1 < 0 || (n0 && !z0) || (n1 && !z1)) return hipErrorInvalidValue;
  const long nbz = (n0 + n1 + 255) / 256;
  const GraphBiasArgs none{};
  hipLaunchKernelGGL(k_embed, dim3((unsigned)(nbe + nbgt + nbz)), dim3(256), 0, s, a, emb, Hout, N, P, rmax, Hs, He, nbe,
                     lat, ga ? *ga : none, ldwc, gout, B, nbg > 0 ? nbg : 1, nbgt, z0, n0, z1, n1);
  return hipGetLastError();
}

__global__ void k_cond_in(const float* __restrict__ temb, int tstride, const int* __restrict__ d_t,
                          const float* __restrict__ text0, const float* __restrict__ text1, int text_dim,
                          float* __restrict__ cin, int B, int P) {
  const int width = TD + text_dim;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)P * B * width) return;
  const long r = idx / width;
  const int k = (int)(idx - r * width);
  const int c = (int)(r / B), gph = (int)(r % B);
  const float* text = c == 0 ? text0 : text1;
  const float* te = d_t ? temb + (long)(*d_t) * TD : temb + (long)gph * tstride;
  cin[idx] = k < TD ? te[k] : text[(long)gph * text_dim + (k - TD)];
}
hipError_t build_cond_in(const float* temb, int tstride, const int* d_t, const float* text0, const float* text1,
                         int text_dim, float* cin, int B, int P, hipStream_t s) {
  const long n = (long)P * B * (TD + text_dim);
  hipLaunchKernelGGL(k_cond_in, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, temb, tstride, d_t, text0, text1,
                     text_dim, cin, B, P);
  return hipGetLastError();
}

__global__ void k_decrement(int* d_t) { *d_t -= 1; }
hipError_t decrement(int* d_t, hipStream_t s) {
  hipLaunchKernelGGL(k_decrement, dim3(1), dim3(1), 0, s, d_t);
  return hipGetLastError();
}

// the per-graph terms of layers beyond the first kGBLayers (blockIdx.y = layer; the first kGBLayers run inside
// k_embed's launch)
__global__ void k_graph_bias(const float* __restrict__ lat, GraphBiasArgs a, long ldwc, float* __restrict__ out, int B) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)B * H) return;
  graph_bias_elem(idx, blockIdx.y, lat, a, ldwc, out, B);
}
hipError_t graph_bias(const float* lat, const GraphBiasArgs& a, int nl, long ldwc, float* out, int B, hipStream_t s) {
  if (nl < 1 || nl > kGBLayers) return hipErrorInvalidValue;
  const long n = (long)B * H;
  hipLaunchKernelGGL(k_graph_bias, dim3((unsigned)((n + 255) / 256), nl), dim3(256), 0, s, lat, a, ldwc, out, B);
  return hipGetLastError();
}

// LayerNorm over 512 features held as 2 x float4 per lane (eps 1e-5, biased variance)
__device__ __forceinline__ void ln512(f32x4& v0, f32x4& v1, const float* w, const float* b, int lane) {
  float s = v0.x + v0.y + v0.z + v0.w + v1.x + v1.y + v1.z + v1.w;
  const float mean = wave_sum(s) * (1.0f / H);
  f32x4 d0 = v0 - mean, d1 = v1 - mean;
  float q = d0.x * d0.x + d0.y * d0.y + d0.z * d0.z + d0.w * d0.w + d1.x * d1.x + d1.y * d1.y + d1.z * d1.z + d1.w * d1.w;
  const float var = wave_sum(q) * (1.0f / H);
  const float rstd = 1.0f / sqrtf(var + 1e-5f);
  const f32x4 w0 = reinterpret_cast<const f32x4*>(w)[lane], w1 = reinterpret_cast<const f32x4*>(w)[64 + lane];
  const f32x4 b0 = reinterpret_cast<const f32x4*>(b)[lane], b1 = reinterpret_cast<const f32x4*>(b)[64 + lane];
  v0 = d0 * rstd * w0 + b0;
  v1 = d1 * rstd * w1 + b1;
}

// FiLM (cspnet.py:78-97) fused with the next CSPLayer's LayerNorm (:175-176):
// Hres = SiLU(LN_f(Y) * scale_g + shift_g) + Hres ; Hl = LN_l(Hres)   (Y null, no FilmLayer: Hl = LN_l(Hres))
__global__ __launch_bounds__(256) void k_film_ln(const float* __restrict__ Y, float* __restrict__ Hres,
                                                 float* __restrict__ Hl, const float* __restrict__ cond_emb,
                                                 const int* __restrict__ n2g, long N, int B, int P,
                                                 const float* fw, const float* fb, const float* lw, const float* lb,
                                                 float* __restrict__ rmx, long rstride, void* Hls, int* Hle) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= N * P) return;
  f32x4* h4 = reinterpret_cast<f32x4*>(Hres + r * H);
  f32x4 v0, v1;
  if (Y) {
    const long c = r / N, i = r - c * N;
    const long crow = c * B + n2g[i];
    const f32x4* y4 = reinterpret_cast<const f32x4*>(Y + r * H);
    v0 = y4[lane];
    v1 = y4[64 + lane];
    ln512(v0, v1, fw, fb, lane);
    const f32x4* sc = reinterpret_cast<const f32x4*>(cond_emb + crow * 2 * H);
    const f32x4* sh = reinterpret_cast<const f32x4*>(cond_emb + crow * 2 * H + H);
    v0 = v0 * sc[lane] + sh[lane];
    v1 = v1 * sc[64 + lane] + sh[64 + lane];
#pragma unroll
    for (int k = 0; k < 4; ++k) { v0[k] = silu(v0[k]); v1[k] = silu(v1[k]); }
    v0 += h4[lane];
    v1 += h4[64 + lane];
    h4[lane] = v0;
    h4[64 + lane] = v1;
  } else {  // (no FilmLayer: Hres passes through)
    v0 = h4[lane];
    v1 = h4[64 + lane];
  }
  ln512(v0, v1, lw, lb, lane);
  f32x4* l4 = reinterpret_cast<f32x4*>(Hl + r * H);
  l4[lane] = v0;
  l4[64 + lane] = v1;
  if (Hls) store_split_row512(v0, v1, lane, Hls, Hle, r);
  if (rmx) {
    float m = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) m = fmaxf(m, fmaxf(fabsf(v0[k]), fabsf(v1[k])));
    m = wave_max(m);
    if (lane == 0) {
      rmx[RMX_HL * rstride + r] = m;
      rmx[RMX_H * rstride + r] = 0.f;
      rmx[RMX_AGG * rstride + r] = 0.f;
      rmx[RMX_U * rstride + r] = 0.f;
    }
  }
}
hipError_t film_ln(const float* Y, float* Hres, float* Hl, const float* cond_emb, const int* n2g, long N, int B, int P,
                   const float* fw, const float* fb, const float* lw, const float* lb, hipStream_t s, float* rmx,
                   long rstride, void* Hls, int* Hle) {
  const long rows = N * P;
  hipLaunchKernelGGL(k_film_ln, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, Y, Hres, Hl, cond_emb, n2g, N, B,
                     P, fw, fb, lw, lb, rmx, rstride, Hls, Hle);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_layer_norm(const float* __restrict__ X, float* __restrict__ Y, long rows,
                                                    const float* w, const float* b) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const f32x4* x4 = reinterpret_cast<const f32x4*>(X + r * H);
  f32x4 v0 = x4[lane], v1 = x4[64 + lane];
  ln512(v0, v1, w, b, lane);
  f32x4* y4 = reinterpret_cast<f32x4*>(Y + r * H);
  y4[lane] = v0;
  y4[64 + lane] = v1;
}
hipError_t layer_norm(const float* X, float* Y, long rows, const float* w, const float* b, hipStream_t s) {
  hipLaunchKernelGGL(k_layer_norm, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, X, Y, rows, w, b);
  return hipGetLastError();
}

// graph mean of final features -> lattice_out (9, no bias) -> (3x3) @ L  (cspnet.py:390-394)
__global__ __launch_bounds__(256) void k_graph_heads(const float* __restrict__ Hf, const float* __restrict__ Wlat,
                                                     const float* __restrict__ lat, const int* __restrict__ node_off,
                                                     const int* __restrict__ natoms, long N, int B,
                                                     float* __restrict__ lat_out) {
  __shared__ float red[4][9];
  __shared__ float l9[9];
  const int c = blockIdx.x / B, gph = blockIdx.x % B;
  const int n = natoms[gph];
  const long r0 = (long)c * N + node_off[gph];
  float part[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) part[q] = 0.f;
  for (int col = threadIdx.x; col < H; col += 256) {
    // the node sum in node order, its loads issued 8 at a time ahead of the adds (one dependent load per node
    // made this a chain of n load latencies: 13.5 us at n = 20)
    float sacc = 0.f;
    const float* hc = Hf + r0 * H + col;
    int k = 0;
    for (; k + 8 <= n; k += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = hc[(long)(k + u) * H];
#pragma unroll
      for (int u = 0; u < 8; ++u) sacc += v[u];
    }
    for (; k < n; ++k) sacc += hc[(long)k * H];
    const float mean = sacc / (float)(n < 1 ? 1 : n);
#pragma unroll
    for (int q = 0; q < 9; ++q) part[q] += Wlat[q * H + col] * mean;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    const float v = wave_sum(part[q]);
    if (lane == 0) red[wv][q] = v;
  }
  __syncthreads();
  if (threadIdx.x < 9) l9[threadIdx.x] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
  __syncthreads();
  if (threadIdx.x < 9) {
    const int a = threadIdx.x / 3, b = threadIdx.x % 3;
    const float* L = lat + gph * 9;
    lat_out[((long)c * B + gph) * 9 + threadIdx.x] = l9[a * 3 + 0] * L[0 * 3 + b] + l9[a * 3 + 1] * L[1 * 3 + b] +
                                                      l9[a * 3 + 2] * L[2 * 3 + b];
  }
}
hipError_t graph_heads(const float* Hf, const float* Wlat, const float* lat, const int* node_off, const int* natoms,
                       long N, int B, int P, float* lat_out, hipStream_t s) {
  hipLaunchKernelGGL(k_graph_heads, dim3((unsigned)(B * P)), dim3(256), 0, s, Hf, Wlat, lat, node_off, natoms, N, B,
                     lat_out);
  return hipGetLastError();
}

__global__ void k_split_heads(const float* __restrict__ HO, long rows, int A, float* types, float* coords) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * (A + 3)) return;
  const long r = idx / (A + 3);
  const int k = (int)(idx - r * (A + 3));
  const float v = HO[r * HEADS_N + k];
  if (k < A) {
    if (types) types[r * A + k] = v;
  } else if (coords) {
    coords[r * 3 + (k - A)] = v;
  }
}
hipError_t split_heads(const float* HO, long rows, int A, float* types, float* coords, hipStream_t s) {
  const long n = rows * (A + 3);
  hipLaunchKernelGGL(k_split_heads, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, HO, rows, A, types, coords);
  return hipGetLastError();
}

__global__ void k_copy_rows(const float* src, long ld_src, float* dst, long ld_dst, long rows, int cols) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * cols) return;
  const long r = idx / cols;
  const int k = (int)(idx - r * cols);
  dst[r * ld_dst + k] = src[r * ld_src + k];
}
hipError_t copy_rows(const float* src, long ld_src, float* dst, long ld_dst, long rows, int cols, hipStream_t s) {
  const long n = rows * cols;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_copy_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, ld_src, dst, ld_dst, rows,
                     cols);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// D3PM reverse sampling (diff_utils.py:258-329). One wave per node; lane d
// holds classes d and d + 64. logits = w1 * L1 + w2 * L2 (classifier-free
// guidance mix, chemeleon.py:288) when L2 != null. fact1 reads the one-step
// matrix at t-1, fact2 the cumulative matrix at t-2 (wrapping to T at t = 1,
// where the result is replaced by the logits), argmax takes the first maximum.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool better(float v, int i, float bv, int bi) {
  const bool vn = v != v, bn = bv != bv;
  if (vn || bn) return vn && (!bn || i < bi);
  return v > bv || (v == bv && i < bi);
}

__global__ __launch_bounds__(256) void k_d3pm(int N, int A, int T, const float* __restrict__ L1, long ld,
                                              const float* __restrict__ L2, float w1, float w2,
                                              const int64_t* __restrict__ xt, const int64_t* __restrict__ tnode,
                                              int t_const, const int* __restrict__ d_t,
                                              const float* __restrict__ noise,
                                              const float* __restrict__ q1, const float* __restrict__ qm,
                                              int64_t* __restrict__ out, uint64_t seed, int64_t node_base,
                                              int* __restrict__ bad) {
  __shared__ float sm_all[4][128];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* sm = sm_all[wv];
  const float eps = 1.0e-6f;
  if (d_t) t_const = *d_t;
  for (long i = (long)blockIdx.x * 4 + wv; i < N; i += (long)gridDim.x * 4) {
    // caller indices (bad != null, chm_d3pm_sample): t outside [1, T] or x_t outside [0, A) records the
    // lowest such node in *bad and writes -1; the sampler's own indices (bad == null) are in range by
    // construction and only clamped, so that nothing can read outside the tables
    const int64_t t_in = tnode ? tnode[i] : (int64_t)t_const, x_in = xt[i];
    if (bad && (t_in < 1 || t_in > T || x_in < 0 || x_in >= A)) {
      if (lane == 0) {
        atomicMin(bad, (int)i);
        out[i] = -1;
      }
      continue;
    }
    const int t = (int)min(max(t_in, (int64_t)1), (int64_t)T);
    const int d0 = lane, d1 = lane + 64;
    const bool ok0 = d0 < A, ok1 = d1 < A;
    float lg0 = ok0 ? L1[i * ld + d0] : -INFINITY;
    float lg1 = ok1 ? L1[i * ld + d1] : -INFINITY;
    if (L2) {
      if (ok0) lg0 = __fadd_rn(__fmul_rn(w1, L2[i * ld + d0]), __fmul_rn(w2, lg0));
      if (ok1) lg1 = __fadd_rn(__fmul_rn(w1, L2[i * ld + d1]), __fmul_rn(w2, lg1));
    }
    // softmax over the A classes
    const float mx = wave_max(fmaxf(lg0, lg1));
    const float e0 = ok0 ? expf(lg0 - mx) : 0.f, e1 = ok1 ? expf(lg1 - mx) : 0.f;
    const float inv = 1.0f / wave_sum(e0 + e1);
    if (ok0) sm[d0] = e0 * inv;
    if (ok1) sm[d1] = e1 * inv;
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    const int x = (int)min(max(x_in, (int64_t)0), (int64_t)(A - 1));
    const long t1 = t - 1;
    const long t2 = (t - 2 + (T + 1)) % (T + 1);
    const float* Q2 = qm + t2 * A * A;
    // sum over cc in order (as one fma chain per class): the Q2 rows of 32 classes are loaded at once,
    // so the loop waits for 4 round trips instead of one per class (71 -> see profiles/r5 at 64x20)
    float f20 = 0.f, f21 = 0.f;
    constexpr int U = 32;
    for (int c0 = 0; c0 < A; c0 += U) {
      float qa[U], qb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int cc = c0 + u;
        qa[u] = (cc < A && ok0) ? Q2[cc * A + d0] : 0.f;
        qb[u] = (cc < A && ok1) ? Q2[cc * A + d1] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int cc = c0 + u;
        if (cc < A) {
          const float p = sm[cc];
          if (ok0) f20 = fmaf(p, qa[u], f20);
          if (ok1) f21 = fmaf(p, qb[u], f21);
        }
      }
    }
    const float* Q1 = q1 + t1 * A * A;
    float v0 = -INFINITY, v1 = -INFINITY;
    const float nz = (t != 1) ? 1.0f : 0.0f;
    if (ok0) {
      float post = (t == 1) ? lg0 : __fadd_rn(logf(Q1[d0 * A + x] + eps), logf(f20 + eps));
      float u = noise ? noise[i * A + d0] : rng_uniform(seed, t, 0, (uint64_t)(i + node_base) * 128 + d0);
      u = fminf(fmaxf(u, eps), 1.0f);
      const float gmb = -logf(-logf(u));
      v0 = __fadd_rn(post, __fmul_rn(gmb, nz));
    }
    if (ok1) {
      float post = (t == 1) ? lg1 : __fadd_rn(logf(Q1[d1 * A + x] + eps), logf(f21 + eps));
      float u = noise ? noise[i * A + d1] : rng_uniform(seed, t, 0, (uint64_t)(i + node_base) * 128 + d1);
      u = fminf(fmaxf(u, eps), 1.0f);
      const float gmb = -logf(-logf(u));
      v1 = __fadd_rn(post, __fmul_rn(gmb, nz));
    }
    float bv = v0;
    int bi = ok0 ? d0 : 1 << 30;
    if (ok1 && better(v1, d1, bv, bi)) { bv = v1; bi = d1; }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) out[i] = bi;
    __builtin_amdgcn_wave_barrier();
  }
}

hipError_t d3pm_sample(int N, int A, int T, const float* logits, long ld_logits, const float* logits2, float w1,
                       float w2, const int64_t* xt, const int64_t* tnode, int t_const, const int* d_t,
                       const float* noise, const float* q1, const float* qm, int64_t* out, uint64_t seed,
                       int64_t node_base, hipStream_t s, int* bad) {
  if (A > 128 || A < 1) return hipErrorInvalidValue;
  long blocks = (N + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k_d3pm, dim3((unsigned)blocks), dim3(256), 0, s, N, A, T, logits, ld_logits, logits2, w1, w2, xt,
                     tnode, t_const, d_t, noise, q1, qm, out, seed, node_base, bad);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// state updates (chemeleon.py:413-437 predictor, :453-462 corrector)
// coef[t] = {c0, c1, sigma_l, step_x, std_x, sqrt_sn, step2, std2}
// ---------------------------------------------------------------------------
__constant__ float c_lat_mask[9] = {1.f, 0.f, 1.f, 1.f, 1.f, 1.f, 0.f, 0.f, 1.f};

__global__ void k_step_predictor(StepArgs a) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (a.d_t) a.t = *a.d_t;
  const float* cf = a.coef + (long)a.t * 8;
  const long nx = a.N * 3;
  if (idx < nx) {
    const long i = idx / 3;
    const int k = (int)(idx - i * 3);
    const long col = a.A + k;
    const float pc = a.HO[i * HEADS_N + col];
    const float pn = a.HO[(a.N + i) * HEADS_N + col];
    const float px = __fadd_rn(__fmul_rn(a.cs_null, pn), __fmul_rn(a.cs_cond, pc));
    float z = 0.f;
    if (a.t > 1) z = a.rx1 ? a.rx1[idx] : rng_normal(a.seed, a.t, 2, (uint64_t)(i + a.node_base) * 3 + k);
    const float pxs = __fmul_rn(px, cf[5]);
    const float xh = __fadd_rn(__fsub_rn(a.x[idx], __fmul_rn(cf[3], pxs)), __fmul_rn(cf[4], z));
    a.x[idx] = xh;
  } else if (idx < nx + (long)a.B * 9) {
    const long r = idx - nx;
    const long gph = r / 9;
    const int q = (int)(r - gph * 9);
    const float pc = a.LAT[r];
    const float pn = a.LAT[(long)a.B * 9 + r];
    const float pl = __fadd_rn(__fmul_rn(a.cs_null, pn), __fmul_rn(a.cs_cond, pc));
    float z = 0.f;
    if (a.t > 1) z = a.rl ? a.rl[r] : rng_normal(a.seed, a.t, 1, (uint64_t)(gph + a.graph_base) * 9 + q);
    const float zm = __fmul_rn(z, c_lat_mask[q]);
    float v = __fadd_rn(__fmul_rn(cf[0], __fsub_rn(a.l[r], __fmul_rn(cf[1], pl))), __fmul_rn(cf[2], zm));
    v = __fmul_rn(v, c_lat_mask[q]);
    if (a.t == a.T) v = v < -6.f ? -6.f : (v > 6.f ? 6.f : v);
    a.l[r] = v;
  }
}

__global__ void k_step_corrector(StepArgs a) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= a.N * 3) return;
  if (a.d_t) a.t = *a.d_t;
  const float* cf = a.coef + (long)a.t * 8;
  const long i = idx / 3;
  const int k = (int)(idx - i * 3);
  const long col = a.A + k;
  const float pc = a.HO[i * HEADS_N + col];
  const float pn = a.HO[(a.N + i) * HEADS_N + col];
  const float px = __fadd_rn(__fmul_rn(a.cs_null, pn), __fmul_rn(a.cs_cond, pc));
  float z = 0.f;
  if (a.t > 1) z = a.rx2 ? a.rx2[idx] : rng_normal(a.seed, a.t, 3, (uint64_t)(i + a.node_base) * 3 + k);
  const float pxs = __fmul_rn(px, cf[5]);
  const float xn = __fadd_rn(__fsub_rn(a.x[idx], __fmul_rn(cf[6], pxs)), __fmul_rn(cf[7], z));
  a.x[idx] = rem1(xn);
}

hipError_t step_predictor(const StepArgs& a, hipStream_t s) {
  const long n = a.N * 3 + (long)a.B * 9;
  hipLaunchKernelGGL(k_step_predictor, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return d3pm_sample((int)a.N, a.A, a.T, a.HO, HEADS_N, a.HO + a.N * HEADS_N, a.cs_null, a.cs_cond, a.a, nullptr,
                     a.t, a.d_t, (a.d_t || a.t > 1) ? a.ra : nullptr, a.q_one_step, a.q_mats, a.a, a.seed,
                     a.node_base, s);
}

hipError_t step_corrector(const StepArgs& a, hipStream_t s) {
  const long n = a.N * 3;
  hipLaunchKernelGGL(k_step_corrector, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Training forward / validation loss (chemeleon.py:137-244): q_sample of the state at per-graph t,
// then (after the decoder) the D3PM hybrid loss, the lattice and coordinate MSEs.
// ---------------------------------------------------------------------------
// d_log_p_wrapped_normal(x, sigma) (diff_utils.py:35-47): 21 wrapped terms, the reference's order
__device__ __forceinline__ float dlogp_wrapped(float x, float s) {
  const float s2 = __fmul_rn(s, s);
  float num = 0.f, den = 0.f;
  for (int i = -10; i <= 10; ++i) {
    const float u = __fadd_rn(x, (float)i);
    const float e = expf(__fdiv_rn(__fdiv_rn(-__fmul_rn(u, u), 2.0f), s2));
    num = __fadd_rn(num, __fmul_rn(__fdiv_rn(u, s2), e));
    den = __fadd_rn(den, e);
  }
  return __fdiv_rn(num, den);
}

// one wave per node: x_t atom type (q_sample: argmax of log(q_mats[t-1][a0] + eps) + Gumbel),
// x_t coordinates ((x0 + sigma z) % 1) and the score target d_log_p(sigma z, sigma) / sqrt(sigma_norm)
__global__ __launch_bounds__(256) void k_train_noise(TrainArgs g) {
  const int lane = threadIdx.x & 63;
  const long i = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= g.N) return;
  const int A = g.A, gph = g.n2g[i];
  const int t = (int)g.t[gph];
  const float eps = 1.0e-6f;
  const int x0 = (int)g.a0[i];
  const float* Q = g.q_mats + ((long)(t - 1) * A + x0) * A;
  float bv = -INFINITY;
  int bi = 0;
  for (int d = lane; d < A; d += 64) {
    const float lg = logf(__fadd_rn(Q[d], eps));
    const float u = fminf(fmaxf(g.rand_a[i * A + d], eps), 1.0f);
    const float v = __fadd_rn(lg, -logf(-logf(u)));
    if (better(v, d, bv, bi)) { bv = v; bi = d; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
  }
  if (lane == 0) g.a_t[i] = bi;
  if (lane < 3) {
    const float* cf = g.coef + (long)t * 4;  // {sqrt(abar), sqrt(1 - abar), sigma_x, sigma_norm}
    const float sz = __fmul_rn(cf[2], g.noise_x[i * 3 + lane]);
    g.x_t[i * 3 + lane] = rem1(__fadd_rn(g.x0[i * 3 + lane], sz));
    g.target_x[i * 3 + lane] = __fdiv_rn(dlogp_wrapped(sz, cf[2]), sqrtf(cf[3]));
  }
}

// l_t = sqrt(abar) l0 + sqrt(1 - abar) noise (noise already masked), one thread per entry
__global__ void k_train_lattice(TrainArgs g) {
  const long k = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (long)g.B * 9) return;
  const float* cf = g.coef + g.t[k / 9] * 4;
  g.l_t[k] = __fadd_rn(__fmul_rn(cf[0], g.l0[k]), __fmul_rn(cf[1], g.noise_l[k]));
}

// one wave per node: true and predicted posterior logits (q_posterior_logits, diff_utils.py:258-286),
// KL(true || pred) (categorical_kl_logits, :288-305) and -log_softmax(pred)[a0] (cross entropy)
__global__ __launch_bounds__(256) void k_train_node_loss(TrainArgs g) {
  __shared__ float sm_all[4][128];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* sm = sm_all[wv];
  const long i = (long)blockIdx.x * 4 + wv;
  if (i >= g.N) return;
  const int A = g.A, T = g.T;
  const int t = (int)g.t[g.n2g[i]];
  const float eps = 1.0e-6f;
  const int x0 = (int)g.a0[i], xt = (int)g.a_t[i];
  const int d0 = lane, d1 = lane + 64;
  const bool ok1 = d1 < A;
  const float* P = g.HO + i * HEADS_N;  // predicted x_0 logits (types head)
  const float lg0 = P[d0], lg1 = ok1 ? P[d1] : -INFINITY;
  // softmax of the prediction
  const float mx = wave_max(fmaxf(lg0, lg1));
  const float e0 = expf(lg0 - mx), e1 = ok1 ? expf(lg1 - mx) : 0.f;
  const float se = wave_sum(e0 + e1);
  sm[d0] = e0 / se;
  if (ok1) sm[d1] = e1 / se;
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  // true x_0 logits: log(one_hot + eps); its softmax row is (1 + eps, eps, ...) normalised
  const float tl0 = logf(__fadd_rn(d0 == x0 ? 1.0f : 0.0f, eps));
  const float tl1 = ok1 ? logf(__fadd_rn(d1 == x0 ? 1.0f : 0.0f, eps)) : -INFINITY;
  float q0 = lg0, q1 = lg1, p0 = tl0, p1 = tl1;  // (t == 1: the x_0 logits themselves)
  if (t != 1) {
    const long t2 = (t - 2 + (T + 1)) % (T + 1);
    const float* Q2 = g.q_mats + t2 * A * A;
    const float* Q1 = g.q_one_step + (long)(t - 1) * A * A;
    // true: softmax(log(onehot + eps)) @ Q2; pred: softmax(pred) @ Q2
    const float tmx = wave_max(fmaxf(tl0, tl1));
    const float te0 = expf(tl0 - tmx), te1 = ok1 ? expf(tl1 - tmx) : 0.f;
    const float tse = wave_sum(te0 + te1);
    float fp0 = 0.f, fp1 = 0.f, ft0 = 0.f, ft1 = 0.f;
    for (int cc = 0; cc < A; ++cc) {
      const float p = sm[cc];
      const float pt = __fdiv_rn(expf(logf(__fadd_rn(cc == x0 ? 1.0f : 0.0f, eps)) - tmx), tse);
      fp0 = fmaf(p, Q2[cc * A + d0], fp0);
      ft0 = fmaf(pt, Q2[cc * A + d0], ft0);
      if (ok1) {
        fp1 = fmaf(p, Q2[cc * A + d1], fp1);
        ft1 = fmaf(pt, Q2[cc * A + d1], ft1);
      }
    }
    const float f10 = logf(__fadd_rn(Q1[d0 * A + xt], eps));
    q0 = __fadd_rn(f10, logf(__fadd_rn(fp0, eps)));
    p0 = __fadd_rn(f10, logf(__fadd_rn(ft0, eps)));
    if (ok1) {
      const float f11 = logf(__fadd_rn(Q1[d1 * A + xt], eps));
      q1 = __fadd_rn(f11, logf(__fadd_rn(fp1, eps)));
      p1 = __fadd_rn(f11, logf(__fadd_rn(ft1, eps)));
    }
  }
  // KL(C(p) || C(q)) with both logits shifted by eps (categorical_kl_logits)
  const float a0 = p0 + eps, a1 = ok1 ? p1 + eps : -INFINITY;
  const float b0 = q0 + eps, b1 = ok1 ? q1 + eps : -INFINITY;
  const float am = wave_max(fmaxf(a0, a1)), bm = wave_max(fmaxf(b0, b1));
  const float ea0 = expf(a0 - am), ea1 = ok1 ? expf(a1 - am) : 0.f;
  const float eb0 = expf(b0 - bm), eb1 = ok1 ? expf(b1 - bm) : 0.f;
  const float lsa = logf(wave_sum(ea0 + ea1)) + am, lsb = logf(wave_sum(eb0 + eb1)) + bm;
  const float sa = wave_sum(ea0 + ea1);
  float kl = (ea0 / sa) * ((a0 - lsa) - (b0 - lsb));
  if (ok1) kl += (ea1 / sa) * ((a1 - lsa) - (b1 - lsb));
  kl = wave_sum(kl);
  // cross entropy of the predicted x_0 logits at a0
  const float lse = logf(se) + mx;
  const float mine = (d0 == x0 ? lg0 : 0.f) + (ok1 && d1 == x0 ? lg1 : 0.f);
  const float ce = lse - wave_sum(mine);
  if (lane == 0) {
    g.part[i * 2 + 0] = kl;
    g.part[i * 2 + 1] = ce;
  }
}

// one block: the means (fixed summation order) and the weighted total
__global__ __launch_bounds__(256) void k_train_reduce(TrainArgs g) {
  __shared__ float red[4][256];
  const int tid = threadIdx.x;
  float kl = 0.f, ce = 0.f, ex = 0.f, el = 0.f;
  for (long i = tid; i < g.N; i += 256) {
    kl += g.part[i * 2];
    ce += g.part[i * 2 + 1];
    for (int k = 0; k < 3; ++k) {
      const float d = g.HO[i * HEADS_N + g.A + k] - g.target_x[i * 3 + k];
      ex += d * d;
    }
  }
  for (long k = tid; k < (long)g.B * 9; k += 256) {
    const int e = (int)(k % 9);
    if (e == 1 || e == 6 || e == 7) continue;  // mask [[1,0,1],[1,1,1],[0,0,1]] (chemeleon.py:70-72)
    const float d = g.LAT[k] - g.noise_l[k];
    el += d * d;
  }
  red[0][tid] = kl; red[1][tid] = ce; red[2][tid] = ex; red[3][tid] = el;
  __syncthreads();
  if (tid < 4) {
    float sacc = 0.f;
    for (int k = 0; k < 256; ++k) sacc += red[tid][k];
    red[tid][0] = sacc;
  }
  __syncthreads();
  if (tid == 0) {
    const float vb = red[0][0] / (float)g.N, cel = red[1][0] / (float)g.N;
    const float lx = red[2][0] / (float)(3 * g.N), ll = red[3][0] / (float)(6 * g.B);
    const float la = vb + cel * g.hybrid;
    g.out[0] = g.cost_a * la + g.cost_l * ll + g.cost_x * lx;
    g.out[1] = vb;
    g.out[2] = cel;
    g.out[3] = la;
    g.out[4] = ll;
    g.out[5] = lx;
  }
}

hipError_t train_noise(const TrainArgs& g, hipStream_t s) {
  hipLaunchKernelGGL(k_train_noise, dim3((unsigned)((g.N + 3) / 4)), dim3(256), 0, s, g);
  hipLaunchKernelGGL(k_train_lattice, dim3((unsigned)((g.B * 9 + 255) / 256)), dim3(256), 0, s, g);
  return hipGetLastError();
}

hipError_t train_loss(const TrainArgs& g, hipStream_t s) {
  hipLaunchKernelGGL(k_train_node_loss, dim3((unsigned)((g.N + 3) / 4)), dim3(256), 0, s, g);
  hipLaunchKernelGGL(k_train_reduce, dim3(1), dim3(256), 0, s, g);
  return hipGetLastError();
}

}  // namespace chm
