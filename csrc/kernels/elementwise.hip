// Memory-bound fused elementwise kernels for gfx950: SwiGLU fwd/bwd, RoPE (in place on the
// packed QKV GEMM output), bias / bias+residual epilogues, bias gradient (column sums).
//
// All use 16-byte vector accesses per lane (8 bf16) and grid-stride loops with grids capped
// at 2048 blocks (Guideline 11: ~256 CUs x 8 blocks).
#include "common.h"

namespace dpfs {

// v_rcp_f32 (1 ulp) instead of an IEEE division (~10 VALU: div_scale / fmas / fixup) per element
__device__ __forceinline__ float silu_f(float g) { return g * __builtin_amdgcn_rcpf(1.f + __expf(-g)); }

static inline int cap_grid(long long work, int block) {
  long long g = (work + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

// ---------------------------------------------------------------------------- SwiGLU --
// gu[M, 2F] = [gate | up]  ->  h[M, F] = silu(gate) * up.   (models/model.py:94-95)
// PERM: gu in the interleaved layout of the fused gate|up epilogue (ops.gemm_select.gu_perm:
// columns [128 b, 128 b + 64) = gate [64 b, 64 b + 64), the next 64 = up of the same columns).
template <bool PERM>
__device__ __forceinline__ long long gate_col(long long c, int F) { return PERM ? ((c >> 6) << 7) + (c & 63) : c; }
template <bool PERM>
__device__ __forceinline__ long long up_col(long long c, int F) { return PERM ? gate_col<true>(c, F) + 64 : F + c; }

template <typename T, bool PERM = false>
__global__ __launch_bounds__(256) void swiglu_fwd_k(const T* __restrict__ gu, T* __restrict__ h, int M, int F) {
  constexpr int N = Vec<T>::N;
  const long long per_row = F / N;
  const long long total = (long long)M * per_row;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / per_row, c = (i % per_row) * N;
    float g[N], u[N], o[N];
    load_vec<T>(gu + r * 2 * F + gate_col<PERM>(c, F), g);
    load_vec<T>(gu + r * 2 * F + up_col<PERM>(c, F), u);
#pragma unroll
    for (int j = 0; j < N; ++j) o[j] = silu_f(g[j]) * u[j];
    store_vec<T>(h + r * F + c, o);
  }
}

// dgu[:, :F] = dh * up * sig(g) * (1 + g (1 - sig(g)));  dgu[:, F:] = dh * silu(g)
template <typename T, bool PERM = false>
__global__ __launch_bounds__(256) void swiglu_bwd_k(const T* __restrict__ dh, const T* __restrict__ gu,
                                                    T* __restrict__ dgu, int M, int F) {
  constexpr int N = Vec<T>::N;
  const long long per_row = F / N;
  const long long total = (long long)M * per_row;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / per_row, c = (i % per_row) * N;
    float g[N], u[N], d[N], og[N], ou[N];
    load_vec<T>(gu + r * 2 * F + gate_col<PERM>(c, F), g);
    load_vec<T>(gu + r * 2 * F + up_col<PERM>(c, F), u);
    load_vec<T>(dh + r * F + c, d);
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const float s = __builtin_amdgcn_rcpf(1.f + __expf(-g[j]));
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

// Same rotation, one 16-byte vector of each half per thread (8 bf16 / 4 fp32 frequency
// pairs) and 32-bit index math: the pass is a pure HBM stream (read + write the q / k
// columns once), where the scalar form above issued 2-byte accesses with 64-bit divisions.
// Needs (hd / 2) % N == 0 and total = M * n_heads * hd / (2 N) < 2^31 (host checks).
template <typename T>
__global__ __launch_bounds__(256) void rope_vec_k(T* __restrict__ qkv, const int64_t* __restrict__ pos,
                                                  const float* __restrict__ table, int M, int ld, int n_heads,
                                                  int hd, float sign) {
  constexpr int N = Vec<T>::N;
  const int h2 = hd / 2;
  const int qn = h2 / N;                 // threads per head
  const int per_row = n_heads * qn;
  const int total = M * per_row;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int row = i / per_row;
    const int rem = i - row * per_row;
    const int head = rem / qn;
    const int f0 = (rem - head * qn) * N;
    KASSERT(pos[row] >= 0, "position %lld at row %d", (long long)pos[row], row);
    const float* tr = table + pos[row] * (long long)hd;
    T* base = qkv + (long long)row * ld + head * hd;
    float x1[N], x2[N], c[N], sn[N];
    load_vec<T>(base + f0, x1);
    load_vec<T>(base + h2 + f0, x2);
#pragma unroll
    for (int j = 0; j < N; j += 4) {
      const f32x4 cv = *reinterpret_cast<const f32x4*>(tr + f0 + j);
      const f32x4 sv = *reinterpret_cast<const f32x4*>(tr + h2 + f0 + j);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        c[j + u] = cv[u];
        sn[j + u] = sign * sv[u];
      }
    }
    float o1[N], o2[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      o1[j] = x1[j] * c[j] - x2[j] * sn[j];
      o2[j] = x2[j] * c[j] + x1[j] * sn[j];
    }
    store_vec<T>(base + f0, o1);
    store_vec<T>(base + h2 + f0, o2);
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

// Column sums (bias gradient, norm-weight gradient partials).  Two deterministic stages,
// both 2-D: a block = 32 column vectors x 8 row lanes, each lane strides over rows, then the
// 8 lanes are reduced through LDS in a fixed order.  Stage 1 reads the bf16/fp32 activation
// grad [M, N] in row chunks -> fp32 partials [R, N]; stage 2 reduces [R, N] -> [N].
template <typename T>
__global__ __launch_bounds__(256) void colsum_stage_k(const T* __restrict__ x, float* __restrict__ out, int M,
                                                      int N_, int rows_per_chunk) {
  constexpr int N = Vec<T>::N;
  __shared__ float red[8][32 * N];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int cvec = blockIdx.x * 32 + tx;
  const int c0 = cvec * N;
  const int r0 = blockIdx.y * rows_per_chunk;
  const int r1 = min(M, r0 + rows_per_chunk);
  float acc[N];
#pragma unroll
  for (int j = 0; j < N; ++j) acc[j] = 0.f;
  if (c0 < N_) {
    for (int r = r0 + ty; r < r1; r += 8) {
      float v[N];
      load_vec<T>(x + (long long)r * N_ + c0, v);
#pragma unroll
      for (int j = 0; j < N; ++j) acc[j] += v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < N; ++j) red[ty][tx * N + j] = acc[j];
  __syncthreads();
  for (int i = threadIdx.x; i < 32 * N; i += 256) {
    const int col = blockIdx.x * 32 * N + i;
    if (col < N_) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) s += red[k][i];
      out[(long long)blockIdx.y * N_ + col] = s;
    }
  }
}

// Stage 2 of every column sum: out[N] = sum over R rows of fp32 partials[R, N].  R is a few
// hundred and N small (768 at GPT-2 width), so the stage-1 shape (32 column vectors per block)
// gave only N/128 blocks of long serial row walks; here a block is 4 column vectors x 64 row
// lanes (N/16 blocks, R/64 rows per lane), reduced through LDS in a fixed order.
// Columns >= split go to out2[col - split] (two column sums reduced by one launch).
template <bool VEC>   // VEC: N % 4 == 0, rows 16-B aligned
__global__ __launch_bounds__(256) void colsum_rows_k(const float* __restrict__ part, float* __restrict__ out, int R,
                                                     int N_, float* __restrict__ out2, int split) {
  __shared__ float red[64][16];
  const int cv = threadIdx.x & 3, rl = threadIdx.x >> 2;
  const int c0 = (blockIdx.x * 4 + cv) * 4;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (c0 < N_) {
    int r = rl;
    if constexpr (VEC) {
      // four rows' vectors in flight per step (the same add order as one at a time: the loads
      // only move ahead of the adds), so the walk is not one load latency per row
      for (; r + 192 < R; r += 256) {
        float v[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) load_vec<float>(part + (long long)(r + 64 * u) * N_ + c0, v[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] += v[u][j];
      }
    }
    for (; r < R; r += 64) {
      const float* p = part + (long long)r * N_ + c0;
      if constexpr (VEC) {
        float v[4];
        load_vec<float>(p, v);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += v[j];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (c0 + j < N_) acc[j] += p[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) red[rl][cv * 4 + j] = acc[j];
  __syncthreads();
  if (threadIdx.x < 16) {
    const int col = blockIdx.x * 16 + threadIdx.x;
    if (col < N_) {
      float s = 0.f;
      for (int k = 0; k < 64; ++k) s += red[k][threadIdx.x];
      if (col < split) out[col] = s;
      else out2[col - split] = s;
    }
  }
}

static inline void colsum_rows(const float* part, float* out, int R, int N_, hipStream_t s, float* out2 = nullptr,
                               int split = -1) {
  if (split < 0) split = N_;
  if (N_ % 4 == 0)
    colsum_rows_k<true><<<dim3((N_ + 15) / 16), 256, 0, s>>>(part, out, R, N_, out2, split);
  else
    colsum_rows_k<false><<<dim3((N_ + 15) / 16), 256, 0, s>>>(part, out, R, N_, out2, split);
}

// Row-chunk plan shared by the fused "elementwise + column-sum" kernels: ~2048 blocks of
// (32 column vectors x 8 row lanes); returns the chunk count, *rpc = rows per chunk.
static int colsum_plan(int M, int cblocks, int target_blocks, int* rpc) {
  int chunks = target_blocks / (cblocks > 0 ? cblocks : 1);
  const int max_chunks = (M + 63) / 64;
  if (chunks > max_chunks) chunks = max_chunks;
  if (chunks < 1) chunks = 1;
  *rpc = (M + chunks - 1) / chunks;
  return (M + *rpc - 1) / *rpc;
}

// SwiGLU backward fused with the gate|up bias gradient: each thread owns one gate column
// vector and its up partner, walks its row chunk, stores dgu and accumulates both column
// sums in fp32; the block's 8 row lanes are reduced through LDS in a fixed order and
// written as partials[chunk][2F] (deterministic; stage 2 = colsum_stage_k<float>).
// (PERM: gu read in the interleaved layout; dgu and the bias-gradient partials are written in
// the natural [gate | up] order, so the data / weight gradient GEMMs use the natural weight.)
template <typename T, bool PERM = false>
__global__ __launch_bounds__(256) void swiglu_bwd_colsum_k(const T* __restrict__ dh, const T* __restrict__ gu,
                                                           T* __restrict__ dgu, float* __restrict__ partial, int M,
                                                           int F, int rows_per_chunk) {
  constexpr int N = Vec<T>::N;
  __shared__ float red[8][2][32 * N];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int c0 = (blockIdx.x * 32 + tx) * N;
  const int r0 = blockIdx.y * rows_per_chunk;
  const int r1 = min(M, r0 + rows_per_chunk);
  float ag[N], au[N];
#pragma unroll
  for (int j = 0; j < N; ++j) ag[j] = au[j] = 0.f;
  if (c0 < F) {
    // Two rows per step (six 16-B loads in flight per thread), same per-thread summation order.
    constexpr int U = 2;
    int r = r0 + ty;
    for (; r < r1; r += 8 * U) {
      float g[U][N], u[U][N], d[U][N];
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const long long rr = r + 8 * q;
        if (q == 0 || rr < r1) {
          load_vec<T>(gu + rr * 2 * F + gate_col<PERM>(c0, F), g[q]);
          load_vec<T>(gu + rr * 2 * F + up_col<PERM>(c0, F), u[q]);
          load_vec<T>(dh + rr * F + c0, d[q]);
        }
      }
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const long long rr = r + 8 * q;
        if (q > 0 && rr >= r1) break;
        float og[N], ou[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
          const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-g[q][j]));
          og[j] = d[q][j] * u[q][j] * sg * (1.f + g[q][j] * (1.f - sg));
          ou[j] = d[q][j] * g[q][j] * sg;
          ag[j] += og[j];
          au[j] += ou[j];
        }
        store_vec<T>(dgu + rr * 2 * F + c0, og);
        store_vec<T>(dgu + rr * 2 * F + F + c0, ou);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    red[ty][0][tx * N + j] = ag[j];
    red[ty][1][tx * N + j] = au[j];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * 32 * N; i += 256) {
    const int half = i / (32 * N), k = i % (32 * N);
    const int col = blockIdx.x * 32 * N + k;
    if (col < F) {
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) sum += red[w][half][k];
      partial[(long long)blockIdx.y * 2 * F + half * F + col] = sum;
    }
  }
}

template <typename T>
static void colsum_launch(const T* x, float* out, float* ws, int M, int N_, hipStream_t s) {
  constexpr int N = Vec<T>::N;
  const int cblocks = (N_ / N + 31) / 32;
  int chunks = 1024 / cblocks;
  const int max_chunks = (M + 63) / 64;
  if (chunks > max_chunks) chunks = max_chunks;
  if (chunks < 1) chunks = 1;
  const int rpc = (M + chunks - 1) / chunks;
  chunks = (M + rpc - 1) / rpc;
  if (chunks == 1) {
    colsum_stage_k<T><<<dim3(cblocks, 1), 256, 0, s>>>(x, out, M, N_, rpc);
    return;
  }
  colsum_stage_k<T><<<dim3(cblocks, chunks), 256, 0, s>>>(x, ws, M, N_, rpc);
  colsum_rows(ws, out, chunks, N_, s);
}

}  // namespace dpfs

using namespace dpfs;

#define PERM_DISPATCH(P, ...) \
  do {                    \
    if (P) {              \
      constexpr bool PM = true; __VA_ARGS__; \
    } else {              \
      constexpr bool PM = false; __VA_ARGS__; \
    }                     \
  } while (0)

extern "C" void dpfs_swiglu_fwd(int dtype, const void* gu, void* h, int M, int F, int perm, hipStream_t s) {
  PERM_DISPATCH(perm, if (dtype == kBF16) swiglu_fwd_k<bf16, PM><<<cap_grid((long long)M * F / 8, 256), 256, 0, s>>>(
                      (const bf16*)gu, (bf16*)h, M, F);
                  else swiglu_fwd_k<float, PM><<<cap_grid((long long)M * F / 4, 256), 256, 0, s>>>(
                      (const float*)gu, (float*)h, M, F));
}

extern "C" void dpfs_swiglu_bwd(int dtype, const void* dh, const void* gu, void* dgu, int M, int F, int perm,
                                hipStream_t s) {
  PERM_DISPATCH(perm, if (dtype == kBF16) swiglu_bwd_k<bf16, PM><<<cap_grid((long long)M * F / 8, 256), 256, 0, s>>>(
                      (const bf16*)dh, (const bf16*)gu, (bf16*)dgu, M, F);
                  else swiglu_bwd_k<float, PM><<<cap_grid((long long)M * F / 4, 256), 256, 0, s>>>(
                      (const float*)dh, (const float*)gu, (float*)dgu, M, F));
}

// Workspace (floats) for dpfs_swiglu_bwd_dbias: partials [chunks, 2F].
extern "C" long long dpfs_swiglu_bwd_dbias_ws(int M, int F) {
  int rpc;
  const int chunks = colsum_plan(M, (F / 8 + 31) / 32, 2048, &rpc);
  return chunks > 1 ? (long long)chunks * 2 * F : 0;
}

extern "C" void dpfs_swiglu_bwd_dbias(int dtype, const void* dh, const void* gu, void* dgu, float* dbias, float* ws,
                                      int M, int F, int perm, hipStream_t s) {
  const int vec = dtype == kBF16 ? 8 : 4;
  const int cblocks = (F / vec + 31) / 32;
  int rpc;
  const int chunks = colsum_plan(M, cblocks, 2048, &rpc);
  float* part = chunks > 1 ? ws : dbias;
  PERM_DISPATCH(perm, if (dtype == kBF16) swiglu_bwd_colsum_k<bf16, PM><<<dim3(cblocks, chunks), 256, 0, s>>>(
                      (const bf16*)dh, (const bf16*)gu, (bf16*)dgu, part, M, F, rpc);
                  else swiglu_bwd_colsum_k<float, PM><<<dim3(cblocks, chunks), 256, 0, s>>>(
                      (const float*)dh, (const float*)gu, (float*)dgu, part, M, F, rpc));
  if (chunks > 1) colsum_rows(ws, dbias, chunks, 2 * F, s);
}

// Stage 2 of a fused column sum: out[N] = sum over `rows` rows of part[rows, N] (fixed order).
extern "C" void dpfs_colsum_rows_small(const float* part, float* out, int rows, int N, hipStream_t s) {
  colsum_rows(part, out, rows, N, s);
}
// ... with columns >= split going to out2 (one launch for two side-by-side column sums).
extern "C" void dpfs_colsum_rows_split(const float* part, float* out, float* out2, int split, int rows, int N,
                                       hipStream_t s) {
  colsum_rows(part, out, rows, N, s, out2, split);
}

extern "C" int dpfs_colsum_plan(int M, int cblocks, int target_blocks, int* rpc) {
  return colsum_plan(M, cblocks, target_blocks, rpc);
}

extern "C" void dpfs_rope(int dtype, void* qkv, const int64_t* pos, const float* table, int M, int ld, int n_heads,
                          int hd, int inverse, hipStream_t s) {
  const long long work = (long long)M * n_heads * (hd / 8);
  const float sign = inverse ? -1.f : 1.f;
  const int vn = dtype == kBF16 ? 8 : 4;
  const long long vwork = (long long)M * n_heads * (hd / 2 / vn);
  if ((hd / 2) % vn == 0 && vwork < (1ll << 31) && ld % vn == 0) {
    const int grid = (int)std::min<long long>((vwork + 255) / 256, 8192);
    if (dtype == kBF16)
      rope_vec_k<bf16><<<grid, 256, 0, s>>>((bf16*)qkv, pos, table, M, ld, n_heads, hd, sign);
    else
      rope_vec_k<float><<<grid, 256, 0, s>>>((float*)qkv, pos, table, M, ld, n_heads, hd, sign);
    return;
  }
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

// Workspace (floats) needed by dpfs_bias_grad / dpfs_colsum_f32 for an [M, N] input.
extern "C" long long dpfs_colsum_ws(int M, int N) { return (long long)((M + 63) / 64) * N; }

extern "C" void dpfs_bias_grad(int dtype, const void* dy, float* out, float* ws, int M, int N, hipStream_t s) {
  if (dtype == kBF16) colsum_launch<bf16>((const bf16*)dy, out, ws, M, N, s);
  else colsum_launch<float>((const float*)dy, out, ws, M, N, s);
}

extern "C" void dpfs_colsum_f32(const float* x, float* out, float* ws, int M, int N, hipStream_t s) {
  colsum_launch<float>(x, out, ws, M, N, s);
}

// Column sums of an fp32 [M, N] whose columns [0, split) go to out and [split, N) to out2:
// two reductions stored side by side in one partial row (the norm backward's weight and
// bias partials) in two launches instead of four.  ws: dpfs_colsum_ws(M, N) floats.
extern "C" void dpfs_colsum_f32_split(const float* x, float* out, float* out2, int split, float* ws, int M, int N,
                                      hipStream_t s) {
  const int cblocks = (N / 4 + 31) / 32;
  int chunks = 1024 / cblocks;
  const int max_chunks = (M + 63) / 64;
  if (chunks > max_chunks) chunks = max_chunks;
  if (chunks < 1) chunks = 1;
  const int rpc = (M + chunks - 1) / chunks;
  chunks = (M + rpc - 1) / rpc;
  colsum_stage_k<float><<<dim3(cblocks, chunks), 256, 0, s>>>(x, ws, M, N, rpc);
  colsum_rows(ws, out, chunks, N, s, out2, split);
}

// ------------------------------------------------------------ collective emulation --
// A stand-in for a TP collective on a side stream (tools/tp_sim.py --emulate-comm, and the
// GEMM co-scheduling tests): `blocks` workgroups of 1024 threads -- the xGMI kernels' grid --
// stay resident for `ticks` of the 100 MHz s_memrealtime clock (each wave sleeps between
// polls, so what it takes from the CU is its residency, as a collective waiting on its peers
// does), then exit.
__global__ __launch_bounds__(1024) void occupy_k(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(16);
}
extern "C" void dpfs_occupy(int blocks, double us, hipStream_t s) {
  if (blocks <= 0 || us <= 0) return;
  occupy_k<<<blocks, 1024, 0, s>>>((unsigned long long)(us * 100.0));
}
