// Fused RMSNorm / LayerNorm forward + backward for gfx950.
//
// Replaces the ~7 ATen kernels per RMSNorm of the reference (float, pow, mean, add, rsqrt,
// mul, type_as, mul: models/layers.py:151-155) and their autograd backward with one pass
// each way.  Layout: x[M, D] row-major, D % (16 B / sizeof(T)) == 0.
//
// Forward: one wave64 per row, the row held in registers (VPL x 16-byte vectors per lane),
// fp32 statistics, 4 rows per 256-thread block.  Memory-bound: 1 read + 1 write of x.
//
// Backward: grid-stride waves over rows; dx per row, and the weight gradient accumulated in
// registers per lane, reduced across the block's 4 waves in a FIXED order through LDS, then
// across blocks by a second column-sum kernel.  No float atomics anywhere: the replicated
// norm weights must get bitwise-identical grads on every TP rank.
#include "common.h"

namespace dpfs {

constexpr int kRowsPerBlock = 4;  // 4 waves

// ------------------------------------------------------------------------- RMSNorm fwd --
template <typename T, int VPL>
__global__ __launch_bounds__(256) void rmsnorm_fwd_k(const T* __restrict__ x, const float* __restrict__ w,
                                                     T* __restrict__ y, float* __restrict__ rstd,
                                                     int M, int D, float eps) {
  constexpr int N = Vec<T>::N;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= M) return;
  const T* xr = x + (size_t)row * D;
  T* yr = y + (size_t)row * D;
  const int nvec = D / N;
  float v[VPL][N];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + i * 64;
    if (c < nvec) {
      load_vec<T>(xr + c * N, v[i]);
#pragma unroll
      for (int j = 0; j < N; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)D + eps);
  if (lane == 0) rstd[row] = r;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + i * 64;
    if (c < nvec) {
      float wv[4 * ((N + 3) / 4)];
      float o[N];
#pragma unroll
      for (int j = 0; j < N; j += 4) {
        f32x4 t = *reinterpret_cast<const f32x4*>(w + c * N + j);
        wv[j] = t[0]; wv[j + 1] = t[1]; wv[j + 2] = t[2]; wv[j + 3] = t[3];
      }
#pragma unroll
      for (int j = 0; j < N; ++j) o[j] = to_f(from_f<T>(v[i][j] * r)) * wv[j];  // reference rounding
      store_vec<T>(yr + c * N, o);
    }
  }
}

// Residual add fused into the norm: xo = y + bias + res (the post-all-reduce epilogue of a
// row-parallel projection), written once; then RMSNorm of the rounded xo.
// Same rounding as bias_residual followed by rmsnorm_fwd.
template <typename T, int VPL>
__global__ __launch_bounds__(256) void add_rmsnorm_fwd_k(const T* __restrict__ yin, const float* __restrict__ bias,
                                                         const T* __restrict__ res, const float* __restrict__ w,
                                                         T* __restrict__ xo, T* __restrict__ y,
                                                         float* __restrict__ rstd, int M, int D, float eps) {
  constexpr int N = Vec<T>::N;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= M) return;
  const size_t off = (size_t)row * D;
  const int nvec = D / N;
  float v[VPL][N];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + i * 64;
    if (c < nvec) {
      float a[N], b[N];
      load_vec<T>(yin + off + c * N, a);
      load_vec<T>(res + off + c * N, b);
#pragma unroll
      for (int j = 0; j < N; ++j) v[i][j] = a[j];
      if (bias) {  // same add order as bias_residual_k: (y + bias) + res
#pragma unroll
        for (int j = 0; j < N; j += 4) {
          const f32x4 t = *reinterpret_cast<const f32x4*>(bias + c * N + j);
          v[i][j] += t[0]; v[i][j + 1] += t[1]; v[i][j + 2] += t[2]; v[i][j + 3] += t[3];
        }
      }
#pragma unroll
      for (int j = 0; j < N; ++j) {
        v[i][j] = to_f(from_f<T>(v[i][j] + b[j]));
        ss += v[i][j] * v[i][j];
      }
      store_vec<T>(xo + off + c * N, v[i]);
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)D + eps);
  if (lane == 0) rstd[row] = r;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + i * 64;
    if (c < nvec) {
      float o[N];
#pragma unroll
      for (int j = 0; j < N; j += 4) {
        const f32x4 t = *reinterpret_cast<const f32x4*>(w + c * N + j);
        o[j] = to_f(from_f<T>(v[i][j] * r)) * t[0];
        o[j + 1] = to_f(from_f<T>(v[i][j + 1] * r)) * t[1];
        o[j + 2] = to_f(from_f<T>(v[i][j + 2] * r)) * t[2];
        o[j + 3] = to_f(from_f<T>(v[i][j + 3] * r)) * t[3];
      }
      store_vec<T>(y + off + c * N, o);
    }
  }
}

// ------------------------------------------------------------------------ LayerNorm fwd --
template <typename T, int VPL>
__global__ __launch_bounds__(256) void layernorm_fwd_k(const T* __restrict__ x, const float* __restrict__ w,
                                                       const float* __restrict__ b, T* __restrict__ y,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd,
                                                       int M, int D, float eps) {
  constexpr int N = Vec<T>::N;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= M) return;
  const T* xr = x + (size_t)row * D;
  T* yr = y + (size_t)row * D;
  const int nvec = D / N;
  float v[VPL][N];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + i * 64;
    if (c < nvec) {
      load_vec<T>(xr + c * N, v[i]);
#pragma unroll
      for (int j = 0; j < N; ++j) s += v[i][j];
    }
  }
  const float mu = wave_sum(s) / (float)D;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + i * 64;
    if (c < nvec) {
#pragma unroll
      for (int j = 0; j < N; ++j) { float d = v[i][j] - mu; ss += d * d; }
    }
  }
  const float r = rsqrtf(wave_sum(ss) / (float)D + eps);
  if (lane == 0) { rstd[row] = r; mean_out[row] = mu; }
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + i * 64;
    if (c < nvec) {
      float o[N];
#pragma unroll
      for (int j = 0; j < N; ++j) o[j] = (v[i][j] - mu) * r * w[c * N + j] + b[c * N + j];
      store_vec<T>(yr + c * N, o);
    }
  }
}

// -------------------------------------------------------------------------- backward --
// MODE 0 = RMSNorm, 1 = LayerNorm, 2 = RMSNorm + column sums of dx.  partial_w: [gridDim.x, D]
// fp32 (MODE 0) or [gridDim.x, 2D] (weight sums then bias / dx sums per row); partial_b unused.
template <typename T, int VPL, int MODE>
__global__ __launch_bounds__(256) void norm_bwd_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                  const float* __restrict__ w, const float* __restrict__ mean_in,
                                                  const float* __restrict__ rstd, const T* __restrict__ dres,
                                                  T* __restrict__ dx, float* __restrict__ partial_w,
                                                  float* __restrict__ partial_b, int M, int D) {
  constexpr int N = Vec<T>::N;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [2][D]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nvec = D / N;
  float aw[VPL][N], ab[VPL][N];
#pragma unroll
  for (int i = 0; i < VPL; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) { aw[i][j] = 0.f; ab[i][j] = 0.f; }

  for (int row = blockIdx.x * kRowsPerBlock + wave; row < M; row += gridDim.x * kRowsPerBlock) {
    const T* xr = x + (size_t)row * D;
    const T* dyr = dy + (size_t)row * D;
    const float r = rstd[row];
    const float mu = MODE == 1 ? mean_in[row] : 0.f;
    float xh[VPL][N], g[VPL][N];
    float dot = 0.f, gs = 0.f;
    // The residual-grad row is loaded with x / dy (packed, 4 VGPRs per vector), not after the
    // row reduction: three loads per lane in flight instead of two plus a dependent one.
    typename Vec<T>::type rvp[VPL];
    if (dres) {
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        const int c = lane + i * 64;
        if (c < nvec) rvp[i] = *reinterpret_cast<const typename Vec<T>::type*>(dres + (size_t)row * D + c * N);
      }
    }
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane + i * 64;
      if (c < nvec) {
        float xv[N], dv[N];
        load_vec<T>(xr + c * N, xv);
        load_vec<T>(dyr + c * N, dv);
#pragma unroll
        for (int j = 0; j < N; ++j) {
          xh[i][j] = (xv[j] - mu) * r;
          g[i][j] = dv[j] * w[c * N + j];
          dot += g[i][j] * xh[i][j];
          gs += g[i][j];
          aw[i][j] += dv[j] * xh[i][j];
          if (MODE == 1) ab[i][j] += dv[j];
        }
      }
    }
    dot = wave_sum(dot) / (float)D;
    if (MODE == 1) gs = wave_sum(gs) / (float)D;
    T* dxr = dx + (size_t)row * D;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane + i * 64;
      if (c < nvec) {
        float o[N];
#pragma unroll
        for (int j = 0; j < N; ++j) o[j] = r * (g[i][j] - (MODE == 1 ? gs : 0.f) - xh[i][j] * dot);
        if (dres) {  // fused residual-stream gradient add (dx += dres)
#pragma unroll
          for (int j = 0; j < N; ++j) o[j] += to_f(rvp[i][j]);
        }
        if (MODE == 2) {  // column sums of the output: the bias grad of the layer below
#pragma unroll
          for (int j = 0; j < N; ++j) ab[i][j] += o[j];
        }
        store_vec<T>(dxr + c * N, o);
      }
    }
  }
  // Deterministic block reduction of the weight grads: waves add in a fixed order.
  for (int wv = 0; wv < kRowsPerBlock; ++wv) {
    if (wave == wv) {
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        const int c = lane + i * 64;
        if (c < nvec) {
#pragma unroll
          for (int j = 0; j < N; ++j) {
            const int col = c * N + j;
            if (wv == 0) {
              red[col] = aw[i][j];
              if (MODE != 0) red[D + col] = ab[i][j];
            } else {
              red[col] += aw[i][j];
              if (MODE != 0) red[D + col] += ab[i][j];
            }
          }
        }
      }
    }
    __syncthreads();
  }
  // Partial row of this block: [D] weight sums, followed for MODE != 0 by the [D] bias sums
  // (one [G, 2D] matrix, reduced by a single two-output column sum).
  const size_t rs = MODE != 0 ? 2 * (size_t)D : (size_t)D;
  for (int col = threadIdx.x; col < D; col += blockDim.x) {
    partial_w[(size_t)blockIdx.x * rs + col] = red[col];
    if (MODE != 0) partial_w[(size_t)blockIdx.x * rs + D + col] = red[D + col];
  }
}

template <typename T>
static int vpl_for(int D) {
  const int nvec = D / Vec<T>::N;
  return (nvec + 63) / 64;
}

#define VPL_DISPATCH(VPL_VALUE, ...)                                   \
  do {                                                                      \
    const int _v = (VPL_VALUE);                                             \
    if (_v <= 1) { constexpr int VPL = 1; __VA_ARGS__; }                    \
    else if (_v <= 2) { constexpr int VPL = 2; __VA_ARGS__; }               \
    else if (_v <= 4) { constexpr int VPL = 4; __VA_ARGS__; }               \
    else if (_v <= 8) { constexpr int VPL = 8; __VA_ARGS__; }               \
    else if (_v <= 12) { constexpr int VPL = 12; __VA_ARGS__; }             \
    else if (_v <= 16) { constexpr int VPL = 16; __VA_ARGS__; }             \
    else if (_v <= 24) { constexpr int VPL = 24; __VA_ARGS__; }             \
    else { constexpr int VPL = 32; __VA_ARGS__; }                           \
  } while (0)

int norm_bwd_grid(int M) {
  int g = (M + kRowsPerBlock - 1) / kRowsPerBlock;
  return g < 1024 ? g : 1024;
}

}  // namespace dpfs

using namespace dpfs;

extern "C" void dpfs_colsum_f32(const float* x, float* out, float* ws, int M, int N, hipStream_t s);
extern "C" void dpfs_colsum_rows_small(const float* part, float* out, int rows, int N, hipStream_t s);
extern "C" void dpfs_colsum_rows_split(const float* part, float* out, float* out2, int split, int rows, int N,
                                       hipStream_t s);
extern "C" void dpfs_colsum_f32_split(const float* x, float* out, float* out2, int split, float* ws, int M, int N,
                                      hipStream_t s);
extern "C" long long dpfs_colsum_ws(int M, int N);

extern "C" int dpfs_norm_bwd_grid(int M) { return norm_bwd_grid(M); }
// Total fp32 workspace of dpfs_norm_bwd: the block partials (x2 for LayerNorm / mode 2).
extern "C" long long dpfs_norm_bwd_ws(int mode, int M, int D) {
  const int G = norm_bwd_grid(M);
  const int cols = D * (mode != 0 ? 2 : 1);
  return (long long)G * cols;
}

extern "C" void dpfs_rmsnorm_fwd(int dtype, const void* x, const float* w, void* y, float* rstd, int M, int D,
                                 float eps, hipStream_t s) {
  dim3 grid((M + kRowsPerBlock - 1) / kRowsPerBlock);
  if (dtype == kBF16) {
    VPL_DISPATCH(vpl_for<bf16>(D), rmsnorm_fwd_k<bf16, VPL><<<grid, 256, 0, s>>>(
        (const bf16*)x, w, (bf16*)y, rstd, M, D, eps));
  } else {
    VPL_DISPATCH(vpl_for<float>(D), rmsnorm_fwd_k<float, VPL><<<grid, 256, 0, s>>>(
        (const float*)x, w, (float*)y, rstd, M, D, eps));
  }
}

extern "C" void dpfs_add_rmsnorm_fwd(int dtype, const void* yin, const float* bias, const void* res, const float* w,
                                     void* xo, void* y, float* rstd, int M, int D, float eps, hipStream_t s) {
  dim3 grid((M + kRowsPerBlock - 1) / kRowsPerBlock);
  if (dtype == kBF16) {
    VPL_DISPATCH(vpl_for<bf16>(D), add_rmsnorm_fwd_k<bf16, VPL><<<grid, 256, 0, s>>>(
        (const bf16*)yin, bias, (const bf16*)res, w, (bf16*)xo, (bf16*)y, rstd, M, D, eps));
  } else {
    VPL_DISPATCH(vpl_for<float>(D), add_rmsnorm_fwd_k<float, VPL><<<grid, 256, 0, s>>>(
        (const float*)yin, bias, (const float*)res, w, (float*)xo, (float*)y, rstd, M, D, eps));
  }
}

extern "C" void dpfs_layernorm_fwd(int dtype, const void* x, const float* w, const float* b, void* y, float* mean,
                                   float* rstd, int M, int D, float eps, hipStream_t s) {
  dim3 grid((M + kRowsPerBlock - 1) / kRowsPerBlock);
  if (dtype == kBF16) {
    VPL_DISPATCH(vpl_for<bf16>(D), layernorm_fwd_k<bf16, VPL><<<grid, 256, 0, s>>>(
        (const bf16*)x, w, b, (bf16*)y, mean, rstd, M, D, eps));
  } else {
    VPL_DISPATCH(vpl_for<float>(D), layernorm_fwd_k<float, VPL><<<grid, 256, 0, s>>>(
        (const float*)x, w, b, (float*)y, mean, rstd, M, D, eps));
  }
}

// mode 0 = rms, 1 = layernorm, 2 = rms + column sums of dx (the bias grad of the layer whose
// output grad dx is) into db.  partial_w: dpfs_norm_bwd_ws floats ([G, D] or [G, 2D] block
// partials, then the column-sum workspace); partial_b is not used (kept for the ABI).
extern "C" void dpfs_norm_bwd(int mode, int dtype, const void* dy, const void* x, const float* w, const float* mean,
                              const float* rstd, const void* dres, void* dx, float* dw, float* db, float* partial_w,
                              float* partial_b, int M, int D, hipStream_t s) {
  const int G = norm_bwd_grid(M);
  const size_t lds = (size_t)(mode != 0 ? 2 : 1) * D * sizeof(float);
#define NB_LAUNCH(T, MODE_)                                                                                  \
  VPL_DISPATCH(vpl_for<T>(D), norm_bwd_k<T, VPL, MODE_><<<G, 256, lds, s>>>(                           \
      (const T*)dy, (const T*)x, w, mean, rstd, (const T*)dres, (T*)dx, partial_w, partial_b, M, D))
  if (dtype == kBF16) {
    if (mode == 0) NB_LAUNCH(bf16, 0); else if (mode == 1) NB_LAUNCH(bf16, 1); else NB_LAUNCH(bf16, 2);
  } else {
    if (mode == 0) NB_LAUNCH(float, 0); else if (mode == 1) NB_LAUNCH(float, 1); else NB_LAUNCH(float, 2);
  }
#undef NB_LAUNCH
  // Stage 2: one fixed-order column reduction of the G (<= 1024) block partials, 64 row lanes
  // per column group (a chunked two-launch reduction cost ~2x its time at these sizes).
  if (mode != 0) dpfs_colsum_rows_split(partial_w, dw, db, D, G, 2 * D, s);
  else dpfs_colsum_rows_small(partial_w, dw, G, D, s);
}
