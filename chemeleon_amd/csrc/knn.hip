// Radius-graph edges of the reference's optional edge_style = "knn" (cspnet.py:325-343), rebuilt on
// the device for every decoder call (the graph depends on the coordinates and lattices):
//
//   k_knn_pairs   one block per crystal: Cartesian positions (einsum of frac and lattice rows), the
//                 smallest interplanar spacing + 0.01 as the radius, every (atom1, atom2, cell) of the
//                 27 neighbouring cells in the reference's order (atom1 major, cell fastest), kept when
//                 r^2 >= d^2 > 1e-4 (radius_graph_pbc, data_utils.py:151-316), compacted in order.
//   k_knn_select  one block per crystal: the neighbour cap (get_max_neighbors_mask, :319-398) -- an atom
//                 with more than max_nb kept pairs keeps those with d^2 below its (max_nb+1)-th
//                 smallest d^2 + 0.01, found by a radix select over the float bits --, then one direction
//                 of every pair (atom2 < atom1, or the same atom with an "earlier" cell) followed by the
//                 reverses (reorder_symmetric_edges, cspnet.py:255-317) with frac_diff = -/+(x2 - x1 + cell),
//                 and each source node's out-degree.
//   (host)        node_estart, segment tiles and E from the degrees (one sync per decoder call).
//   k_knn_place   edges grouped by source node, in their order within each node (a stable sort: the
//                 per-node sums of the fused scatter_mean then follow scatter_add's order).
//
// All arithmetic is fp32 with explicitly rounded operations in the reference's expression order; the
// reference runs these as ATen CPU kernels, so a pair within an ulp of the radius can differ (the tests
// treat pairs that close to the cut as undecided).
#include "chm_internal.h"

namespace chm {

namespace {

// exclusive prefix of a flag over the 256 threads of the block (4 waves), plus the block total
__device__ __forceinline__ int block_scan_flag(bool f, int* w4, int& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long bal = __ballot(f);
  const int pre = __popcll(bal & ((1ull << lane) - 1ull));
  if (lane == 0) w4[w] = __popcll(bal);
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int v = w4[k];
    if (k < w) off += v;
    tot += v;
  }
  __syncthreads();
  total = tot;
  return off + pre;
}

// u of cell c (meshgrid 'ij' of [-1, 0, 1]^3, last axis fastest; data_utils.py:234-242)
__device__ __forceinline__ float cell_u(int c, int ax) {
  return (float)((ax == 0 ? c / 9 : ax == 1 ? (c / 3) % 3 : c % 3) - 1);
}

// cell "earlier" than its mirror (cspnet.py:276-283)
__device__ __forceinline__ bool cell_earlier(int c) {
  const int u0 = c / 9 - 1, u1 = (c / 3) % 3 - 1, u2 = c % 3 - 1;
  return u0 < 0 || (u0 == 0 && u1 < 0) || (u0 == 0 && u1 == 0 && u2 < 0);
}

__device__ __forceinline__ void cross3(const float* a, const float* b, float* o) {
  o[0] = __fsub_rn(__fmul_rn(a[1], b[2]), __fmul_rn(a[2], b[1]));
  o[1] = __fsub_rn(__fmul_rn(a[2], b[0]), __fmul_rn(a[0], b[2]));
  o[2] = __fsub_rn(__fmul_rn(a[0], b[1]), __fmul_rn(a[1], b[0]));
}

// 1 / || (a x b) / vol ||  (data_utils.py:202-219)
__device__ __forceinline__ float inv_spacing(const float* a, const float* b, float vol) {
  float c[3];
  cross3(a, b, c);
  const float v0 = __fdiv_rn(c[0], vol), v1 = __fdiv_rn(c[1], vol), v2 = __fdiv_rn(c[2], vol);
  const float nrm = __fsqrt_rn(__fadd_rn(__fadd_rn(__fmul_rn(v0, v0), __fmul_rn(v1, v1)), __fmul_rn(v2, v2)));
  return __fdiv_rn(1.0f, nrm);
}

}  // namespace

__global__ __launch_bounds__(256) void k_knn_pairs(KnnArgs g) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const int n = g.natoms[b], o = g.node_off[b];
  const long base = g.cand_off[b];
  __shared__ float pos[256][3];
  __shared__ float off[27][3];
  __shared__ float r2s;
  __shared__ int cnt[256];
  __shared__ int w4[4];
  const float* L = g.lat + (long)b * 9;
  if (tid == 0) {
    float c23[3];
    cross3(L + 3, L + 6, c23);
    const float vol = __fadd_rn(__fadd_rn(__fmul_rn(L[0], c23[0]), __fmul_rn(L[1], c23[1])), __fmul_rn(L[2], c23[2]));
    const float d1 = inv_spacing(L + 3, L + 6, vol), d2 = inv_spacing(L + 6, L + 0, vol), d3 = inv_spacing(L + 0, L + 3, vol);
    const float r = __fadd_rn(fminf(fminf(d1, d2), d3), 0.01f);
    r2s = __fmul_rn(r, r);
  }
  if (tid < 81) {  // offsets of the 27 cells: bmm(cell^T, u), k = 0, 1, 2 in order
    const int c = tid / 3, ax = tid % 3;
    off[c][ax] = __fadd_rn(__fadd_rn(__fmul_rn(L[ax], cell_u(c, 0)), __fmul_rn(L[3 + ax], cell_u(c, 1))),
                           __fmul_rn(L[6 + ax], cell_u(c, 2)));
  }
  for (int a = tid; a < n; a += 256) {  // einsum("bi,bij->bj"): sum over i in order
    const float* xa = g.x + (long)(o + a) * 3;
#pragma unroll
    for (int j = 0; j < 3; ++j)
      pos[a][j] = __fadd_rn(__fadd_rn(__fmul_rn(xa[0], L[j]), __fmul_rn(xa[1], L[3 + j])), __fmul_rn(xa[2], L[6 + j]));
    cnt[a] = 0;
  }
  __syncthreads();
  const float r2 = r2s;
  const long total = (long)n * n * 27;
  long run = 0;
  for (long c0 = 0; c0 < total; c0 += 256) {
    const long idx = c0 + tid;
    bool keep = false;
    unsigned key = 0;
    float d2 = 0.f;
    if (idx < total) {
      const int i = (int)(idx / (n * 27)), rem = (int)(idx % (n * 27)), j = rem / 27, c = rem % 27;
      const float dx = __fsub_rn(pos[i][0], __fadd_rn(pos[j][0], off[c][0]));
      const float dy = __fsub_rn(pos[i][1], __fadd_rn(pos[j][1], off[c][1]));
      const float dz = __fsub_rn(pos[i][2], __fadd_rn(pos[j][2], off[c][2]));
      d2 = __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
      keep = d2 <= r2 && d2 > 0.0001f;
      key = ((unsigned)i << 16) | ((unsigned)j << 8) | (unsigned)c;
    }
    int tot;
    const int p = block_scan_flag(keep, w4, tot);
    if (keep) {
      g.cand_key[base + run + p] = key;
      g.cand_d2[base + run + p] = d2;
      atomicAdd(&cnt[key >> 16], 1);
    }
    run += tot;
  }
  __syncthreads();
  for (int a = tid; a < n; a += 256) g.atom_cnt[o + a] = cnt[a];
}

__global__ __launch_bounds__(256) void k_knn_select(KnnArgs g) {
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = g.natoms[b], o = g.node_off[b];
  const long base = g.cand_off[b];
  __shared__ int start[257], nstart[257];
  __shared__ int kept[256], deg[256];
  __shared__ float cutv[256];
  __shared__ unsigned hist[4][256];
  __shared__ int sel[4][2];
  __shared__ int w4[4];
  for (int a = tid; a < n; a += 256) {
    kept[a] = g.atom_cnt[o + a];
    deg[a] = 0;
  }
  __syncthreads();
  if (tid == 0) {
    int s = 0;
    for (int a = 0; a < n; ++a) {
      start[a] = s;
      s += kept[a];
    }
    start[n] = s;
  }
  __syncthreads();
  // the neighbour cap: one wave per atom, uniform trip count (barriers inside)
  const int thr = g.max_nb;
  for (int a0 = 0; a0 < n; a0 += 4) {
    const int a = a0 + wave;
    const bool act = a < n;
    const int c = act ? start[a + 1] - start[a] : 0;
    const float* d2 = g.cand_d2 + base + (act ? start[a] : 0);
    const bool capped = act && thr > 0 && c > thr;
    // radix select of the thr-th smallest (0-based) d^2 among the atom's pairs: d^2 >= 0, so the
    // float bits order as unsigned integers
    unsigned prefix = 0, mask = 0;
    int k = thr;
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int q = lane; q < 256; q += 64) hist[wave][q] = 0;
      __syncthreads();
      if (capped)
        for (int e = lane; e < c; e += 64) {
          const unsigned u = __float_as_uint(d2[e]);
          if ((u & mask) == prefix) atomicAdd(&hist[wave][(u >> shift) & 255u], 1u);
        }
      __syncthreads();
      if (capped && lane == 0) {
        int cum = 0, dgt = 255;
        for (int q = 0; q < 256; ++q) {
          const int h = (int)hist[wave][q];
          if (cum + h > k) {
            dgt = q;
            break;
          }
          cum += h;
        }
        sel[wave][0] = dgt;
        sel[wave][1] = k - cum;
      }
      __syncthreads();
      if (capped) {
        prefix |= (unsigned)sel[wave][0] << shift;
        mask |= 255u << shift;
        k = sel[wave][1];
      }
    }
    // keep d^2 < v + 0.01 (all pairs of an atom at or below the cap)
    const float cut = capped ? __fadd_rn(__uint_as_float(prefix), 0.01f) : __int_as_float(0x7f800000);
    int cntk = 0;
    if (act)
      for (int e = lane; e < c; e += 64) cntk += d2[e] < cut ? 1 : 0;
    for (int s2 = 32; s2 > 0; s2 >>= 1) cntk += __shfl_xor(cntk, s2, 64);
    if (act && lane == 0) {
      kept[a] = cntk;
      cutv[a] = cut;
    }
  }
  __syncthreads();
  if (tid == 0) {
    int s = 0;
    for (int a = 0; a < n; ++a) {
      nstart[a] = s;
      s += kept[a];
    }
    nstart[n] = s;
  }
  __syncthreads();
  // compaction of every atom's kept pairs, in order (wave per atom)
  for (int a = wave; a < n; a += 4) {
    const int c = start[a + 1] - start[a];
    const float cut = cutv[a];
    int run = 0;
    for (int e0 = 0; e0 < c; e0 += 64) {
      const int e = e0 + lane;
      const bool keep = e < c && g.cand_d2[base + start[a] + e] < cut;
      const unsigned long long bal = __ballot(keep);
      if (keep) g.cand2[base + nstart[a] + run + __popcll(bal & ((1ull << lane) - 1ull))] = g.cand_key[base + start[a] + e];
      run += __popcll(bal);
    }
  }
  __syncthreads();
  // one direction of every pair, then the reverses: first pass counts, second writes
  const int K = nstart[n];
  int D = 0;
  for (int pass = 0; pass < 2; ++pass) {
    int run = 0;
    for (int e0 = 0; e0 < K; e0 += 256) {
      const int e = e0 + tid;
      bool dir = false;
      unsigned key = 0;
      if (e < K) {
        key = g.cand2[base + e];
        const int i = key >> 16, j = (key >> 8) & 255, c = key & 255;
        dir = j < i || (j == i && cell_earlier(c));
      }
      int tot;
      const int p = block_scan_flag(dir, w4, tot);
      if (pass == 1 && dir) {
        const int i = key >> 16, j = (key >> 8) & 255, c = key & 255;
        const long f0 = 2 * base + run + p, f1 = 2 * base + D + run + p;
        g.fin_key[f0] = ((unsigned)j << 8) | (unsigned)i;  // (src, dst) = (atom2, atom1)
        g.fin_key[f1] = ((unsigned)i << 8) | (unsigned)j;  // the reverse
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) {  // ev = x2 - x1 + cell; frac_diff = -ev, then +ev (cspnet.py:331-343)
          const float ev = __fadd_rn(__fsub_rn(g.x[(long)(o + j) * 3 + ax], g.x[(long)(o + i) * 3 + ax]), cell_u(c, ax));
          g.fin_fd[f0 * 3 + ax] = -ev;
          g.fin_fd[f1 * 3 + ax] = ev;
        }
        atomicAdd(&deg[j], 1);
        atomicAdd(&deg[i], 1);
      }
      run += tot;
    }
    if (pass == 0) D = run;
  }
  __syncthreads();
  for (int a = tid; a < n; a += 256) g.deg[o + a] = deg[a];
  if (tid == 0) g.cryst_fin[b] = 2 * D;
}

// edges of crystal b grouped by source node, in list order within a node (a stable sort by source)
__global__ __launch_bounds__(256) void k_knn_place(KnnArgs g) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const int n = g.natoms[b], o = g.node_off[b];
  const long base2 = 2 * g.cand_off[b];
  const int F = g.cryst_fin[b];
  __shared__ long cur[256];
  __shared__ unsigned short srcs[256];
  for (int a = tid; a < n; a += 256) cur[a] = g.node_estart[o + a];
  __syncthreads();
  for (int e0 = 0; e0 < F; e0 += 256) {
    const int e = e0 + tid;
    unsigned key = 0;
    int src = -1;
    if (e < F) {
      key = g.fin_key[base2 + e];
      src = (int)(key >> 8);
      srcs[tid] = (unsigned short)src;
    }
    __syncthreads();
    long pos = 0;
    if (e < F) {
      int r = 0;
      for (int q = 0; q < tid; ++q) r += srcs[q] == src;
      pos = cur[src] + r;
      g.ei[pos] = o + src;
      g.ej[pos] = o + (int)(key & 255u);
#pragma unroll
      for (int ax = 0; ax < 3; ++ax) g.fd[pos * 3 + ax] = g.fin_fd[(base2 + e) * 3 + ax];
    }
    __syncthreads();
    if (e < F) atomicAdd(reinterpret_cast<unsigned long long*>(&cur[src]), 1ull);
    __syncthreads();
  }
}

hipError_t knn_candidates(const KnnArgs& g, int B, hipStream_t s) {
  hipLaunchKernelGGL(k_knn_pairs, dim3(B), dim3(256), 0, s, g);
  hipLaunchKernelGGL(k_knn_select, dim3(B), dim3(256), 0, s, g);
  return hipGetLastError();
}

hipError_t knn_place(const KnnArgs& g, int B, hipStream_t s) {
  hipLaunchKernelGGL(k_knn_place, dim3(B), dim3(256), 0, s, g);
  return hipGetLastError();
}

}  // namespace chm
