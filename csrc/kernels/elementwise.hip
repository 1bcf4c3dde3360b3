// Memory-bound fused elementwise kernels for gfx950: SwiGLU fwd/bwd, RoPE (in place on the
// packed QKV GEMM output), bias / bias+residual epilogues, bias gradient (column sums).
//
// All use 16-byte vector accesses per lane (8 bf16) and grid-stride loops with grids capped
// at 2048 blocks (Guideline 11: ~256 CUs x 8 blocks).
#include "common.h"

namespace dpfs {

__device__ __forceinline__ float silu_f(float g) { return g / (1.f + __expf(-g)); }

static inline int cap_grid(long long work, int block) {
  long long g = (work + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

// ---------------------------------------------------------------------------- SwiGLU --
// gu[M, 2F] = [gate | up]  ->  h[M, F] = silu(gate) * up.   (models/model.py:94-95)
template <typename T>
__global__ __launch_bounds__(256) void swiglu_fwd_k(const T* __restrict__ gu, T* __restrict__ h, int M, int F) {
  constexpr int N = Vec<T>::N;
  const long long per_row = F / N;
  const long long total = (long long)M * per_row;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / per_row, c = (i % per_row) * N;
    float g[N], u[N], o[N];
    load_vec<T>(gu + r * 2 * F + c, g);
    load_vec<T>(gu + r * 2 * F + F + c, u);
#pragma unroll
    for (int j = 0; j < N; ++j) o[j] = silu_f(g[j]) * u[j];
    store_vec<T>(h + r * F + c, o);
  }
}

// dgu[:, :F] = dh * up * sig(g) * (1 + g (1 - sig(g)));  dgu[:, F:] = dh * silu(g)
template <typename T>
__global__ __launch_bounds__(256) void swiglu_bwd_k(const T* __restrict__ dh, const T* __restrict__ gu,
                                                    T* __restrict__ dgu, int M, int F) {
  constexpr int N = Vec<T>::N;
  const long long per_row = F / N;
  const long long total = (long long)M * per_row;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / per_row, c = (i % per_row) * N;
    float g[N], u[N], d[N], og[N], ou[N];
    load_vec<T>(gu + r * 2 * F + c, g);
    load_vec<T>(gu + r * 2 * F + F + c, u);
    load_vec<T>(dh + r * F + c, d);
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const float s = 1.f / (1.f + __expf(-g[j]));
      og[j] = d[j] * u[j] * s * (1.f + g[j] * (1.f - s));
      ou[j] = d[j] * g[j] * s;
    }
    store_vec<T>(dgu + r * 2 * F + c, og);
    store_vec<T>(dgu + r * 2 * F + F + c, ou);
  }
}

// ------------------------------------------------------------------------------ RoPE --
// In place on qkv[M, ld]: the first n_heads heads of each row (q then k heads) are rotated
// by the angle of positions[row] (rotate-half convention, models/model.py:17-31):
//   o1 = x1 c - x2 s,  o2 = x2 c + x1 s   (sign = -1 for the inverse / backward rotation).
// table[maxlen, hd] fp32 = [cos(p f_0..f_{h2-1}) | sin(...)].  Each thread owns 4 frequency
// pairs (two 8-byte bf16x4 accesses).
template <typename T>
__global__ __launch_bounds__(256) void rope_k(T* __restrict__ qkv, const int64_t* __restrict__ pos,
                                              const float* __restrict__ table, int M, int ld, int n_heads,
                                              int hd, float sign) {
  const int h2 = hd / 2;
  const int q4 = h2 / 4;  // threads per head
  const long long total = (long long)M * n_heads * q4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long row = i / (n_heads * q4);
    const int rem = (int)(i % (n_heads * q4));
    const int head = rem / q4;
    const int f0 = (rem % q4) * 4;
    const float* tr = table + pos[row] * (long long)hd;
    T* base = qkv + row * (long long)ld + (long long)head * hd;
    float c[4], sn[4], x1[4], x2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c[j] = tr[f0 + j];
      sn[j] = sign * tr[h2 + f0 + j];
      x1[j] = to_f(base[f0 + j]);
      x2[j] = to_f(base[h2 + f0 + j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      base[f0 + j] = from_f<T>(x1[j] * c[j] - x2[j] * sn[j]);
      base[h2 + f0 + j] = from_f<T>(x2[j] * c[j] + x1[j] * sn[j]);
    }
  }
}

// ------------------------------------------------------------------- bias / residual --
// out = (residual ? residual : 0) + y + bias  (bias may be null; out may alias y).
template <typename T>
__global__ __launch_bounds__(256) void bias_residual_k(const T* __restrict__ y, const float* __restrict__ bias,
                                                       const T* __restrict__ res, T* out, int M, int N_) {
  constexpr int N = Vec<T>::N;
  const long long per_row = N_ / N;
  const long long total = (long long)M * per_row;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / per_row, c = (i % per_row) * N;
    float v[N];
    load_vec<T>(y + r * N_ + c, v);
    if (bias) {
#pragma unroll
      for (int j = 0; j < N; ++j) v[j] += bias[c + j];
    }
    if (res) {
      float rv[N];
      load_vec<T>(res + r * N_ + c, rv);
#pragma unroll
      for (int j = 0; j < N; ++j) v[j] += rv[j];
    }
    store_vec<T>(out + r * N_ + c, v);
  }
}

// Bias gradient: column sums of dy[M, N] -> fp32 partials [G, N] (each block a contiguous
// row range, fixed order), then a fixed-order reduction over G.  Deterministic.
template <typename T>
__global__ __launch_bounds__(256) void colsum_rows_k(const T* __restrict__ dy, float* __restrict__ partial,
                                                     int M, int N_, int rows_per_block) {
  constexpr int N = Vec<T>::N;
  const int nvec = N_ / N;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < nvec; c += gridDim.x * blockDim.x) {
    float acc[N];
#pragma unroll
    for (int j = 0; j < N; ++j) acc[j] = 0.f;
    for (int r = r0; r < r1; ++r) {
      float v[N];
      load_vec<T>(dy + (long long)r * N_ + c * N, v);
#pragma unroll
      for (int j = 0; j < N; ++j) acc[j] += v[j];
    }
#pragma unroll
    for (int j = 0; j < N; ++j) partial[(long long)blockIdx.y * N_ + c * N + j] = acc[j];
  }
}

__global__ __launch_bounds__(256) void colsum_final_k(const float* __restrict__ partial, float* __restrict__ out,
                                                      int G, int N_) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= N_) return;
  float s = 0.f;
  for (int g = 0; g < G; ++g) s += partial[(long long)g * N_ + c];
  out[c] = s;
}

}  // namespace dpfs

using namespace dpfs;

extern "C" void dpfs_swiglu_fwd(int dtype, const void* gu, void* h, int M, int F, hipStream_t s) {
  if (dtype == kBF16)
    swiglu_fwd_k<bf16><<<cap_grid((long long)M * F / 8, 256), 256, 0, s>>>((const bf16*)gu, (bf16*)h, M, F);
  else
    swiglu_fwd_k<float><<<cap_grid((long long)M * F / 4, 256), 256, 0, s>>>((const float*)gu, (float*)h, M, F);
}

extern "C" void dpfs_swiglu_bwd(int dtype, const void* dh, const void* gu, void* dgu, int M, int F, hipStream_t s) {
  if (dtype == kBF16)
    swiglu_bwd_k<bf16><<<cap_grid((long long)M * F / 8, 256), 256, 0, s>>>((const bf16*)dh, (const bf16*)gu,
                                                                              (bf16*)dgu, M, F);
  else
    swiglu_bwd_k<float><<<cap_grid((long long)M * F / 4, 256), 256, 0, s>>>((const float*)dh, (const float*)gu,
                                                                               (float*)dgu, M, F);
}

extern "C" void dpfs_rope(int dtype, void* qkv, const int64_t* pos, const float* table, int M, int ld, int n_heads,
                          int hd, int inverse, hipStream_t s) {
  const long long work = (long long)M * n_heads * (hd / 8);
  const float sign = inverse ? -1.f : 1.f;
  if (dtype == kBF16)
    rope_k<bf16><<<cap_grid(work, 256), 256, 0, s>>>((bf16*)qkv, pos, table, M, ld, n_heads, hd, sign);
  else
    rope_k<float><<<cap_grid(work, 256), 256, 0, s>>>((float*)qkv, pos, table, M, ld, n_heads, hd, sign);
}

extern "C" void dpfs_bias_residual(int dtype, const void* y, const float* bias, const void* res, void* out, int M,
                                   int N, hipStream_t s) {
  if (dtype == kBF16)
    bias_residual_k<bf16><<<cap_grid((long long)M * N / 8, 256), 256, 0, s>>>((const bf16*)y, bias, (const bf16*)res,
                                                                                (bf16*)out, M, N);
  else
    bias_residual_k<float><<<cap_grid((long long)M * N / 4, 256), 256, 0, s>>>((const float*)y, bias,
                                                                                 (const float*)res, (float*)out, M, N);
}

extern "C" int dpfs_colsum_groups(int M) {
  int g = (M + 255) / 256;  // 256 rows per block
  return g < 1 ? 1 : g;
}

extern "C" void dpfs_bias_grad(int dtype, const void* dy, float* out, float* partial, int M, int N, hipStream_t s) {
  const int G = dpfs_colsum_groups(M);
  const int rows = (M + G - 1) / G;
  const int vecN = dtype == kBF16 ? 8 : 4;
  dim3 grid((N / vecN + 255) / 256, G);
  if (dtype == kBF16)
    colsum_rows_k<bf16><<<grid, 256, 0, s>>>((const bf16*)dy, partial, M, N, rows);
  else
    colsum_rows_k<float><<<grid, 256, 0, s>>>((const float*)dy, partial, M, N, rows);
  colsum_final_k<<<(N + 255) / 256, 256, 0, s>>>(partial, out, G, N);
}
