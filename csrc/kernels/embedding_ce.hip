// Vocab-sharded embedding (fwd/bwd) and vocab-parallel cross-entropy kernels for gfx950.
//
// Embedding forward fuses the reference's 5 kernels (two compares + logical_and, two
// index_put_ on the *caller's* ids, F.embedding, index_put of zeros: models/layers.py:137-140)
// and the bf16 cast (models/model.py:153-154) into one gather: one wave per token row,
// 16-byte loads of the fp32 master row, bf16 stores; ids outside [vocab_start, vocab_start
// + V_local) produce zeros.  The ids are never written.
//
// Embedding backward: scatter-add of the output-grad rows into the fp32 table shard with
// no-return global_atomic_add_f32, shaped as the guide asks (each wave-instruction = 256
// contiguous bytes of one row; rows spread over the table).
//
// Cross-entropy: per-row online max / sum-exp over the local shard in ONE pass (fp32), the
// target logit if owned; backward writes (softmax - onehot) * g in place over the logits.
#include "common.h"

namespace dpfs {

template <typename TO>
__global__ __launch_bounds__(256) void embedding_fwd_k(const int64_t* __restrict__ ids, const float* __restrict__ w,
                                                       TO* __restrict__ out, int M, int D, long long vstart,
                                                       int vlocal) {
  const int lane = threadIdx.x & 63;
  const int nv = D / 4;
  for (int row = blockIdx.x * 4 + (threadIdx.x >> 6); row < M; row += gridDim.x * 4) {
    KASSERT(ids[row] >= 0, "token id %lld at row %d", (long long)ids[row], row);
    const long long loc = ids[row] - vstart;
    const bool hit = loc >= 0 && loc < vlocal;
    TO* o = out + (long long)row * D;
    for (int c = lane; c < nv; c += 64) {
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (hit) v = *reinterpret_cast<const f32x4*>(w + loc * D + c * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[c * 4 + j] = from_f<TO>(v[j]);
    }
  }
}

template <typename TI>
__global__ __launch_bounds__(256) void embedding_bwd_k(const TI* __restrict__ dout, const int64_t* __restrict__ ids,
                                                       float* __restrict__ dw, int M, int D, long long vstart,
                                                       int vlocal) {
  const int lane = threadIdx.x & 63;
  for (int row = blockIdx.x * 4 + (threadIdx.x >> 6); row < M; row += gridDim.x * 4) {
    KASSERT(ids[row] >= 0, "token id %lld at row %d", (long long)ids[row], row);
    const long long loc = ids[row] - vstart;
    if (loc < 0 || loc >= vlocal) continue;
    const TI* g = dout + (long long)row * D;
    float* dst = dw + loc * D;
    for (int c = lane; c < D; c += 64) atomicAdd(dst + c, to_f(g[c]));
  }
}

// ------------------------------------------------------------------- cross entropy ----
struct MaxSum {
  float m, s;
};
__device__ __forceinline__ MaxSum merge(MaxSum a, MaxSum b) {
  const float m = fmaxf(a.m, b.m);
  if (m == -INFINITY) return {m, 0.f};
  return {m, a.s * __expf(a.m - m) + b.s * __expf(b.m - m)};
}

// One 256-thread block per row.  stats[row] = {max, sum exp(x - max), target logit or 0}.
template <typename T>
__global__ __launch_bounds__(256) void ce_stats_k(const T* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                  float* __restrict__ stats, int V, long long vstart, int vvalid) {
  constexpr int N = Vec<T>::N;
  __shared__ MaxSum red[4];
  const int row = blockIdx.x;
  const T* x = logits + (long long)row * V;
  MaxSum acc = {-INFINITY, 0.f};
  // full vectors inside the valid range (rows are 16-B aligned only when V % N == 0)
  const int nvec = V % N == 0 ? vvalid / N : 0;
  for (int c = threadIdx.x; c < nvec; c += blockDim.x) {
    float v[N];
    load_vec<T>(x + c * N, v);
    float m = v[0];
#pragma unroll
    for (int j = 1; j < N; ++j) m = fmaxf(m, v[j]);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < N; ++j) s += __expf(v[j] - m);
    acc = merge(acc, {m, s});
  }
  for (int c = nvec * N + threadIdx.x; c < vvalid; c += blockDim.x) acc = merge(acc, {to_f(x[c]), 1.f});
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    MaxSum other = {__shfl_xor(acc.m, o, 64), __shfl_xor(acc.s, o, 64)};
    acc = merge(acc, other);
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    MaxSum r = red[0];
    for (int i = 1; i < 4; ++i) r = merge(r, red[i]);
    KASSERT(tgt[row] >= -1, "target %lld at row %d (ignore_index is -1)", (long long)tgt[row], row);
    const long long loc = tgt[row] - vstart;
    const float tl = (loc >= 0 && loc < vvalid) ? to_f(x[loc]) : 0.f;
    stats[row * 3 + 0] = r.m;
    stats[row * 3 + 1] = r.s;
    stats[row * 3 + 2] = tl;
  }
}

// N-wide access: the 16-byte vector when N == Vec<T>::N, element-wise otherwise (rows whose
// width is not a multiple of the vector, e.g. an uneven vocab shard, are not 16-B aligned).
template <typename T, int N>
__device__ __forceinline__ void load_n(const T* p, float (&out)[N]) {
  if constexpr (N == Vec<T>::N) {
    load_vec<T>(p, out);
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = to_f(p[i]);
  }
}
template <typename T, int N>
__device__ __forceinline__ void store_n(T* p, const float (&in)[N]) {
  if constexpr (N == Vec<T>::N) {
    store_vec<T>(p, in);
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) p[i] = from_f<T>(in[i]);
  }
}

// out[row, c] = (exp(x - lse[row]) - [c == target]) * g[row]; 0 for c >= vvalid.  out may
// alias logits (in place).
template <typename T, int N>
__global__ __launch_bounds__(256) void ce_bwd_k(const T* logits, const int64_t* __restrict__ tgt,
                                                const float* __restrict__ lse, const float* __restrict__ gscale,
                                                T* out, int M, int V, long long vstart, int vvalid) {
  const long long per_row = V / N;
  const long long total = (long long)M * per_row;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / per_row;
    const int c = (int)(i % per_row) * N;
    const float l = lse[r], g = gscale[r];
    const long long loc = tgt[r] - vstart;
    float v[N];
    load_n<T, N>(logits + r * V + c, v);
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const int col = c + j;
      float p = col < vvalid ? __expf(v[j] - l) : 0.f;
      if (col == loc && col < vvalid) p -= 1.f;
      v[j] = p * g;
    }
    store_n<T, N>(out + r * V + c, v);
  }
}

// CE backward fused with the lm_head bias gradient (column sums of dlogits): 2-D blocks of
// 32 column vectors x 8 row lanes over a row chunk; fp32 partials [chunk][V], reduced in a
// fixed order (deterministic).  Saves one full re-read of the [M, V_local] logits.
template <typename T, int N>
__global__ __launch_bounds__(256) void ce_bwd_colsum_k(const T* logits, const int64_t* __restrict__ tgt,
                                                       const float* __restrict__ lse,
                                                       const float* __restrict__ gscale, T* out,
                                                       float* __restrict__ partial, int M, int V, long long vstart,
                                                       int vvalid, int rows_per_chunk) {
  __shared__ float red[8][32 * N];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int c = (blockIdx.x * 32 + tx) * N;
  const int r0 = blockIdx.y * rows_per_chunk;
  const int r1 = min(M, r0 + rows_per_chunk);
  float acc[N];
#pragma unroll
  for (int j = 0; j < N; ++j) acc[j] = 0.f;
  if (c < V) {
    // 8 rows per step: eight independent 16-B loads in flight per thread before the first use
    // (one row at a time left the kernel latency-bound; 4 -> 8 rows: 1341 -> 1299 us per
    // GPT-2-small step at 117 VGPRs, 4 waves per SIMD).
    constexpr int U = 8;
    int r = r0 + ty;
    for (; r + 8 * (U - 1) < r1; r += 8 * U) {
      float v[U][N];
#pragma unroll
      for (int u = 0; u < U; ++u) load_n<T, N>(logits + (long long)(r + 8 * u) * V + c, v[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int ru = r + 8 * u;
        const float l = lse[ru], g = gscale[ru];
        const long long loc = tgt[ru] - vstart;
#pragma unroll
        for (int j = 0; j < N; ++j) {
          const int col = c + j;
          float p = col < vvalid ? __expf(v[u][j] - l) : 0.f;
          if (col == loc && col < vvalid) p -= 1.f;
          v[u][j] = p * g;
          acc[j] += v[u][j];
        }
        store_n<T, N>(out + (long long)ru * V + c, v[u]);
      }
    }
    for (; r < r1; r += 8) {
      const float l = lse[r], g = gscale[r];
      const long long loc = tgt[r] - vstart;
      float v[N];
      load_n<T, N>(logits + (long long)r * V + c, v);
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const int col = c + j;
        float p = col < vvalid ? __expf(v[j] - l) : 0.f;
        if (col == loc && col < vvalid) p -= 1.f;
        v[j] = p * g;
        acc[j] += v[j];
      }
      store_n<T, N>(out + (long long)r * V + c, v);
    }
  }
#pragma unroll
  for (int j = 0; j < N; ++j) red[ty][tx * N + j] = acc[j];
  __syncthreads();
  for (int i = threadIdx.x; i < 32 * N; i += 256) {
    const int col = blockIdx.x * 32 * N + i;
    if (col < V) {
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) sum += red[w][i];
      partial[(long long)blockIdx.y * V + col] = sum;
    }
  }
}

static inline int cap_grid2(long long work, int block) {
  long long g = (work + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace dpfs

using namespace dpfs;

extern "C" int dpfs_colsum_plan(int M, int cblocks, int target_blocks, int* rpc);
extern "C" void dpfs_colsum_rows_small(const float* part, float* out, int rows, int N, hipStream_t s);

// Vector width of the CE backward: 16 B when every row is 16-B aligned, else element-wise.
static inline int ce_vec(int dtype, int V) {
  const int w = dtype == kBF16 ? 8 : 4;
  return V % w == 0 ? w : 1;
}

extern "C" long long dpfs_ce_bwd_dbias_ws(int dtype, int M, int V) {
  int rpc;
  const int chunks = dpfs_colsum_plan(M, (V / ce_vec(dtype, V) + 31) / 32, 2048, &rpc);
  return chunks > 1 ? (long long)chunks * V : 0;
}

extern "C" void dpfs_ce_bwd_dbias(int dtype, const void* logits, const int64_t* tgt, const float* lse,
                                  const float* gscale, void* out, float* dbias, float* ws, int M, int V,
                                  long long vstart, int vvalid, hipStream_t s) {
  const int vec = ce_vec(dtype, V);
  const int cblocks = (V / vec + 31) / 32;
  int rpc;
  const int chunks = dpfs_colsum_plan(M, cblocks, 2048, &rpc);
  float* part = chunks > 1 ? ws : dbias;
  const dim3 grid(cblocks, chunks);
  if (dtype == kBF16 && vec == 8)
    ce_bwd_colsum_k<bf16, 8><<<grid, 256, 0, s>>>((const bf16*)logits, tgt, lse, gscale, (bf16*)out, part, M, V,
                                                  vstart, vvalid, rpc);
  else if (dtype == kBF16)
    ce_bwd_colsum_k<bf16, 1><<<grid, 256, 0, s>>>((const bf16*)logits, tgt, lse, gscale, (bf16*)out, part, M, V,
                                                  vstart, vvalid, rpc);
  else if (vec == 4)
    ce_bwd_colsum_k<float, 4><<<grid, 256, 0, s>>>((const float*)logits, tgt, lse, gscale, (float*)out, part, M, V,
                                                   vstart, vvalid, rpc);
  else
    ce_bwd_colsum_k<float, 1><<<grid, 256, 0, s>>>((const float*)logits, tgt, lse, gscale, (float*)out, part, M, V,
                                                   vstart, vvalid, rpc);
  if (chunks > 1) dpfs_colsum_rows_small(ws, dbias, chunks, V, s);
}

extern "C" void dpfs_embedding_fwd(int out_dtype, const int64_t* ids, const float* w, void* out, int M, int D,
                                   long long vstart, int vlocal, hipStream_t s) {
  const int grid = cap_grid2(M, 4);
  if (out_dtype == kBF16)
    embedding_fwd_k<bf16><<<grid, 256, 0, s>>>(ids, w, (bf16*)out, M, D, vstart, vlocal);
  else
    embedding_fwd_k<float><<<grid, 256, 0, s>>>(ids, w, (float*)out, M, D, vstart, vlocal);
}

// dw must be zeroed by the caller.
extern "C" void dpfs_embedding_bwd(int in_dtype, const void* dout, const int64_t* ids, float* dw, int M, int D,
                                   long long vstart, int vlocal, hipStream_t s) {
  const int grid = cap_grid2(M, 4);
  if (in_dtype == kBF16)
    embedding_bwd_k<bf16><<<grid, 256, 0, s>>>((const bf16*)dout, ids, dw, M, D, vstart, vlocal);
  else
    embedding_bwd_k<float><<<grid, 256, 0, s>>>((const float*)dout, ids, dw, M, D, vstart, vlocal);
}

extern "C" void dpfs_ce_stats(int dtype, const void* logits, const int64_t* tgt, float* stats, int M, int V,
                              long long vstart, int vvalid, hipStream_t s) {
  if (M == 0) return;
  if (dtype == kBF16)
    ce_stats_k<bf16><<<M, 256, 0, s>>>((const bf16*)logits, tgt, stats, V, vstart, vvalid);
  else
    ce_stats_k<float><<<M, 256, 0, s>>>((const float*)logits, tgt, stats, V, vstart, vvalid);
}

extern "C" void dpfs_ce_bwd(int dtype, const void* logits, const int64_t* tgt, const float* lse, const float* gscale,
                            void* out, int M, int V, long long vstart, int vvalid, hipStream_t s) {
  const int vec = ce_vec(dtype, V);
  const int grid = cap_grid2((long long)M * V / vec, 256);
  if (dtype == kBF16 && vec == 8)
    ce_bwd_k<bf16, 8><<<grid, 256, 0, s>>>((const bf16*)logits, tgt, lse, gscale, (bf16*)out, M, V, vstart, vvalid);
  else if (dtype == kBF16)
    ce_bwd_k<bf16, 1><<<grid, 256, 0, s>>>((const bf16*)logits, tgt, lse, gscale, (bf16*)out, M, V, vstart, vvalid);
  else if (vec == 4)
    ce_bwd_k<float, 4><<<grid, 256, 0, s>>>((const float*)logits, tgt, lse, gscale, (float*)out, M, V, vstart,
                                            vvalid);
  else
    ce_bwd_k<float, 1><<<grid, 256, 0, s>>>((const float*)logits, tgt, lse, gscale, (float*)out, M, V, vstart,
                                            vvalid);
}
