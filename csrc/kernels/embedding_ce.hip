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

#include <algorithm>

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

// Deterministic form (no atomics): the rows sorted by token id (stable: ascending row order
// within an id) and each vocab row's segment [seg[v], seg[v + 1]) of the sorted order; one wave
// per vocab row sums its segment's gradient rows in that fixed order and WRITES the row (zeros
// for an id no row carries), or adds it to dw (`accumulate`: the later ping-pong chunks) -- no
// zero pass, run-to-run bit-identical.  Four rows' vectors in flight per step.
template <typename TI>
__device__ __forceinline__ void load4f(const TI* p, float (&x)[4]) {
  if constexpr (sizeof(TI) == 2) {
    typedef TI t4 __attribute__((ext_vector_type(4)));
    const t4 v = *reinterpret_cast<const t4*>(p);
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = to_f(v[k]);
  } else {
    const f32x4 v = *reinterpret_cast<const f32x4*>(p);
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = v[k];
  }
}
template <typename TI>
__global__ __launch_bounds__(256) void embedding_bwd_seg_k(const TI* __restrict__ dout, const int64_t* __restrict__ perm,
                                                           const int64_t* __restrict__ seg, float* __restrict__ dw,
                                                           int D, int vlocal, int accumulate) {
  const int lane = threadIdx.x & 63;
  for (int v = blockIdx.x * 4 + (threadIdx.x >> 6); v < vlocal; v += gridDim.x * 4) {
    const long long s0 = seg[v], e0 = seg[v + 1];
    float* dst = dw + (long long)v * D;
    for (int c = lane * 4; c < D; c += 256) {
      f32x4 acc = accumulate ? *reinterpret_cast<const f32x4*>(dst + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      long long j = s0;
      for (; j + 3 < e0; j += 4) {
        float x[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) load4f<TI>(dout + perm[j + u] * D + c, x[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[k] += x[u][k];
      }
      for (; j < e0; ++j) {
        float x[4];
        load4f<TI>(dout + perm[j] * D + c, x);
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] += x[k];
      }
      *reinterpret_cast<f32x4*>(dst + c) = acc;
    }
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

// Single-shard CE forward + backward in ONE pass over the logits (TP 1: the row's lse is
// local, so d logits can be written during the forward; reference train.py:101-104 computes
// the loss on gathered logits and backward re-reads them).  The two-pass form (ce_stats_k,
// then ce_bwd_colsum_k in backward) reads the 3.3 GB of GPT-2-small logits twice and writes
// them once; this one reads once and writes once:
//   * one 512-thread workgroup per CU (2 waves per SIMD: 256 registers for the row's NV
//     vectors and their 8 NV fp32 column sums) walks rows r = blockIdx.x + k * gridDim.x;
//   * a row (V bf16, V % 8 == 0, V <= 8 * 512 * NV) arrives in LDS by LDS-DMA, lane-linear:
//     vector c = 512 i + t lands at byte 16 c, written AND later read by thread t only, so no
//     barrier guards the staging; thread t moves its NV vectors into registers, then issues the
//     DMA of its slots of the NEXT row (same bytes: its own reads retired first), which lands
//     while this row is reduced, differentiated and stored;
//   * one exponential per element: e = exp(x - m_i) against its 16-byte vector's max m_i,
//     summed in fp32 and kept as fp16 pairs in place of the bf16 input (e <= 1); after the
//     block reduction (per thread -> wave xor butterfly -> 8 waves through LDS, double-
//     buffered by row parity: one barrier per row) p = e * exp(m_i - lse) * gscale[row]
//     (- gscale at the target), in place as bf16, 0 past vvalid;
//   * the row's stores are buffer stores issued by every lane (out-of-range lanes past the
//     descriptor), NV per wave, so the next row's entry wait leaves exactly them in flight
//     (vmcnt(NV): the next row's DMA, issued before them, has landed);
//   * the lm_head bias gradient: each thread sums its fixed columns over its rows in fp32;
//     one partial row per workgroup (part[blockIdx.x][V]), reduced by colsum_rows.
// stats[row] = {max, sum exp(x - max), target logit or 0} as ce_stats_k.
template <int NV>
__global__ __launch_bounds__(512) void ce_fused_k(bf16* logits, const int64_t* __restrict__ tgt,
                                                   const float* __restrict__ gscale, float* __restrict__ stats,
                                                   float* __restrict__ part, int M, int V, long long vstart,
                                                   int vvalid) {
  __shared__ __attribute__((aligned(1024))) char row_lds[NV * 8192];
  __shared__ MaxSum red[2][8];
  constexpr float L2E = 1.4426950408889634f;
  const int t = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nvec = V >> 3;
  const unsigned row_bytes = (unsigned)V * 2u;
  float acc[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[i][e] = 0.f;
  auto rsrc = [&](int row) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(logits + (long long)row * V), (short)0, (int)row_bytes,
                                             0x00020000);
  };
  // byte offset of slot i's vector in a row (past the descriptor for the last slot's spare lanes)
  auto voff = [&](int i) -> unsigned {
    const int c = 512 * i + t;
    return (i < NV - 1 || c < nvec) ? (unsigned)c * 16u : kOOB;
  };
  auto issue = [&](int row) {
    const __amdgpu_buffer_rsrc_t r = rsrc(row);
#pragma unroll
    for (int i = 0; i < NV; ++i) dma16(r, row_lds + i * 8192 + wave * 1024, voff(i));
  };
  // bf16 -> fp32 of slot i, -inf past vvalid (by opaque shifts / masks: hipcc would otherwise
  // keep fp32 copies or hoist per-element masks out of the row loop, both spilling)
  auto elems = [&](const u32x4& w, int i, float (&x)[8]) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      unsigned lo, hi;
      asm volatile("v_lshlrev_b32 %0, 16, %2\n\tv_and_b32 %1, 0xffff0000, %2" : "=&v"(lo), "=&v"(hi) : "v"(w[h]));
      x[2 * h] = __builtin_bit_cast(float, lo);
      x[2 * h + 1] = __builtin_bit_cast(float, hi);
    }
    if (8 * 512 * (i + 1) > vvalid) {
      int nv;   // valid elements of this vector (<= 0: none)
      asm volatile("v_sub_u32 %0, %1, %2" : "=v"(nv) : "s"(vvalid), "v"(8 * (512 * i + t)));
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = e < nv ? x[e] : -INFINITY;
    }
  };
  int row = blockIdx.x;
  if (row < M) issue(row);
  for (int it = 0; row < M; row += gridDim.x, ++it) {
    if (it == 0) wait_vmcnt<0>();
    else wait_vmcnt<NV>();   // this row's DMA landed; the previous row's NV stores may be in flight
    u32x4 cur[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) cur[i] = *reinterpret_cast<const u32x4*>(row_lds + (512 * i + t) * 16);
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this thread's LDS reads retired
    const int nrow = row + gridDim.x;
    if (nrow < M) issue(nrow);
    KASSERT(tgt[row] >= -1, "target %lld at row %d (ignore_index is -1)", (long long)tgt[row], row);
    const long long loc64 = tgt[row] - vstart;
    const int loc = (loc64 >= 0 && loc64 < vvalid) ? (int)loc64 : -1;   // target column in this shard
    // per slot: its max m_i, e = exp(x - m_i) as fp16 pairs in place (e <= 1), the slot's sum
    // merged into the thread's (max, sum)
    float mi[NV];
    MaxSum ms = {-INFINITY, 0.f};
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      float x[8];
      elems(cur[i], i, x);
      const int d = loc - 8 * (512 * i + t);
      if ((unsigned)d < 8u) {
        float tl = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) tl = e == d ? x[e] : tl;
        stats[row * 3 + 2] = tl;
      }
      float m = x[0];
#pragma unroll
      for (int e = 1; e < 8; ++e) m = fmaxf(m, x[e]);
      mi[i] = m;
      const float ms_ = m == -INFINITY ? 0.f : m * L2E;
      float sm = 0.f;
      u32x4 ev;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const float e0 = __builtin_amdgcn_exp2f(x[2 * h] * L2E - ms_);
        const float e1 = __builtin_amdgcn_exp2f(x[2 * h + 1] * L2E - ms_);
        sm += e0 + e1;
        // (packed by opaque asm: hipcc would otherwise keep each fp16 in a register of its own)
        unsigned pk, tmp;
        asm volatile("v_cvt_f16_f32 %0, %2\n\tv_cvt_f16_f32 %1, %3\n\tv_pack_b32_f16 %0, %0, %1"
                     : "=&v"(pk), "=&v"(tmp) : "v"(e0), "v"(e1));
        ev[h] = pk;
      }
      cur[i] = ev;
      if (m != -INFINITY) ms = merge(ms, {m, sm});
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ms = merge(ms, {__shfl_xor(ms.m, o, 64), __shfl_xor(ms.s, o, 64)});
    if ((t & 63) == 0) red[it & 1][wave] = ms;
    __syncthreads();
    MaxSum r = red[it & 1][0];
#pragma unroll
    for (int w = 1; w < 8; ++w) r = merge(r, red[it & 1][w]);
    if (t == 0) {
      stats[row * 3 + 0] = r.m;
      stats[row * 3 + 1] = r.s;
      if (loc < 0) stats[row * 3 + 2] = 0.f;
    }
    // p = e * exp(m_i - lse) * g  (g = 0 on ignored rows; a slot with no valid column has e = 0)
    const float g = gscale[row];
    const float lse2 = r.m * L2E + __log2f(r.s);
    const __amdgpu_buffer_rsrc_t ro = rsrc(row);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const float sc = mi[i] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mi[i] * L2E - lse2) * g;
      float p[8];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        float lo, hi;
        asm volatile("v_cvt_f32_f16 %0, %2\n\tv_lshrrev_b32 %1, 16, %2\n\tv_cvt_f32_f16 %1, %1"
                     : "=&v"(lo), "=&v"(hi) : "v"(cur[i][h]));
        p[2 * h] = lo * sc;
        p[2 * h + 1] = hi * sc;
      }
      const int d = loc - 8 * (512 * i + t);
      if ((unsigned)d < 8u) {
#pragma unroll
        for (int e = 0; e < 8; ++e) p[e] = e == d ? p[e] - g : p[e];
      }
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        acc[i][e] += p[e];
        o[e] = (bf16)p[e];
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), ro, voff(i), 0, 0);
    }
  }
  if (part != nullptr) {
    float* pr = part + (long long)blockIdx.x * V;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = 512 * i + t;
      if (i == NV - 1 && c >= nvec) continue;
      *reinterpret_cast<f32x4*>(pr + 8 * c) = (f32x4){acc[i][0], acc[i][1], acc[i][2], acc[i][3]};
      *reinterpret_cast<f32x4*>(pr + 8 * c + 4) = (f32x4){acc[i][4], acc[i][5], acc[i][6], acc[i][7]};
    }
  }
}

static inline int cap_grid2(long long work, int block) {
  long long g = (work + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}


// ---------------------------------------------------------------- CE loss bookkeeping --
// The loss scalar and per-row terms of the vocab-parallel CE from the gathered statistics
// (replaces ~15 small framework kernels per step: amax / log / exp / where / sums / casts).
// Rows are split over kCeBlocks workgroups that write (loss, count) partials; a one-workgroup
// pass adds them in block order.  Every sum has a fixed order, so the loss is run-to-run
// bit-identical.
//   stats (nsh, M, 3) = {max, sum exp(x - max), target logit or 0} per vocab shard;
//   lse[r] = mx + log(sum_s se_s exp(m_s - mx)); valid[r] = (tgt[r] != ignore) as 1.0 / 0.0;
//   acc[0] (+)= sum valid (lse - tl), acc[1] (+)= sum valid; with `last`: acc[1] = max(acc[1], 1),
//   loss = acc[0] / acc[1].
constexpr int kCeBlocks = 64;

// fixed-order block sum of (a, b) over 256 threads; thread 0 gets the totals
__device__ __forceinline__ void block_sum2(float& a, float& b) {
  __shared__ float red[2][256];
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = b;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      red[0][threadIdx.x] += red[0][threadIdx.x + o];
      red[1][threadIdx.x] += red[1][threadIdx.x + o];
    }
    __syncthreads();
  }
  a = red[0][0];
  b = red[1][0];
}

__global__ __launch_bounds__(256) void ce_finalize_rows_k(const float* __restrict__ stats,
                                                          const int64_t* __restrict__ tgt, long long ignore,
                                                          float* __restrict__ lse, float* __restrict__ valid,
                                                          float* __restrict__ part, int M, int nsh) {
  float ls = 0.f, cn = 0.f;
  const int per = (M + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * per, r1 = min(M, r0 + per);
  for (int r = r0 + threadIdx.x; r < r1; r += 256) {
    float mx = -INFINITY;
    for (int sh = 0; sh < nsh; ++sh) mx = fmaxf(mx, stats[((long long)sh * M + r) * 3]);
    float se = 0.f, tl = 0.f;
    for (int sh = 0; sh < nsh; ++sh) {
      const float* st = stats + ((long long)sh * M + r) * 3;
      se += st[1] * __expf(st[0] - mx);
      tl += st[2];
    }
    const float l = mx + __logf(se);
    const float v = tgt[r] != ignore ? 1.f : 0.f;
    lse[r] = l;
    valid[r] = v;
    ls += v != 0.f ? l - tl : 0.f;
    cn += v;
  }
  block_sum2(ls, cn);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = ls;
    part[2 * blockIdx.x + 1] = cn;
  }
}

__global__ __launch_bounds__(64) void ce_finalize_sum_k(const float* __restrict__ part, int nb,
                                                        float* __restrict__ acc, float* __restrict__ loss, int first,
                                                        int last) {
  if (threadIdx.x != 0) return;
  float a0 = 0.f, a1 = 0.f;
  for (int b = 0; b < nb; ++b) {
    a0 += part[2 * b];
    a1 += part[2 * b + 1];
  }
  if (!first) {
    a0 += acc[0];
    a1 += acc[1];
  }
  if (last) {
    a1 = fmaxf(a1, 1.f);
    loss[0] = a0 / a1;
  }
  acc[0] = a0;
  acc[1] = a1;
}

// gs[r] = (tgt[r] != ignore) / max(count, 1) over all M rows (the one-pass TP-1 CE's per-row
// gradient scale for a unit loss gradient); n_valid[0] = max(count, 1).  Per-block counts, then
// every block adds them in block order and writes its rows.
__global__ __launch_bounds__(256) void ce_valid_count_k(const int64_t* __restrict__ tgt, long long ignore,
                                                        float* __restrict__ part, int M) {
  float cn = 0.f, z = 0.f;
  const int per = (M + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * per, r1 = min(M, r0 + per);
  for (int r = r0 + threadIdx.x; r < r1; r += 256) cn += tgt[r] != ignore ? 1.f : 0.f;
  block_sum2(cn, z);
  if (threadIdx.x == 0) part[blockIdx.x] = cn;
}
__global__ __launch_bounds__(256) void ce_valid_scale_k(const int64_t* __restrict__ tgt, long long ignore,
                                                        const float* __restrict__ part, float* __restrict__ gs,
                                                        float* __restrict__ n_valid, int M) {
  float n = 0.f;
  for (int b = 0; b < (int)gridDim.x; ++b) n += part[b];
  n = fmaxf(n, 1.f);
  const float inv = 1.f / n;
  const int per = (M + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * per, r1 = min(M, r0 + per);
  for (int r = r0 + threadIdx.x; r < r1; r += 256) gs[r] = tgt[r] != ignore ? inv : 0.f;
  if (blockIdx.x == 0 && threadIdx.x == 0) n_valid[0] = n;
}

// d loss / d row of the CE backward: gs[r] = valid[r] * gloss / n_valid (gloss: the loss's
// incoming gradient, fp32 or bf16 scalar; n_valid: the fp32 valid-row count of ce_finalize), one
// launch instead of a framework divide + multiply.
template <typename TG>
__global__ __launch_bounds__(256) void ce_grad_scale_k(const float* __restrict__ valid, const TG* __restrict__ gloss,
                                                       const float* __restrict__ n_valid, float* __restrict__ gs, int M) {
  const float c = (float)gloss[0] / n_valid[0];
  for (int r = blockIdx.x * 256 + threadIdx.x; r < M; r += gridDim.x * 256) gs[r] = valid[r] * c;
}

// --------------------------------------------- deterministic counting sort of token ids --
// The deterministic embedding backward needs the ids' stable order and each local vocab row's
// segment (perm, seg).  A two-pass LSD radix sort on 8-bit digits of the 16-bit key (local id,
// or 0xFFFF for an id outside this vocab shard), chunks of 1024 tokens (one 1024-thread
// workgroup each), stable: within a wave the rank among equal digits comes from ballots (the
// match mask of the 8 digit bits), across the 16 waves from per-wave digit counts in LDS, across
// chunks from the (digit, chunk) count table.  Per pass: emb_digit_hist_k writes the chunk's 256
// counts (no zeroing, no atomics), emb_digit_scatter_k derives the chunk's global offsets from
// the whole table and moves (key, token) pairs; emb_seg_k then finds every row's segment start
// by binary search.  Replaces the framework's sort + searchsorted (rocprim + ATen kernels).
constexpr int kSortChunk = 1024;

// rank of this lane among the active lanes of its wave with the same 8-bit digit, and the
// mask of those lanes
__device__ __forceinline__ unsigned long long digit_match(int d, bool active) {
  unsigned long long m = __builtin_amdgcn_ballot_w64(active);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const bool bit = (d >> b) & 1;
    const unsigned long long bal = __builtin_amdgcn_ballot_w64(bit);
    m &= bit ? bal : ~bal;
  }
  return m;
}

// Per-wave digit counts of the chunk into LDS wc[16][256] (zeroed here), then each thread
// t < 256 turns column t into an exclusive prefix over the waves; returns the chunk total of
// digit threadIdx.x (threads < 256).
__device__ __forceinline__ int chunk_digit_prefix(int (&wc)[16][256], int d, bool active, unsigned long long m) {
  for (int i = threadIdx.x; i < 16 * 256; i += 1024) (&wc[0][0])[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  if (active && (m & lt) == 0) wc[w][d] = __popcll(m);   // the first lane of each digit group
  __syncthreads();
  int tot = 0;
  if (threadIdx.x < 256) {
    for (int ww = 0; ww < 16; ++ww) {
      const int c = wc[ww][threadIdx.x];
      wc[ww][threadIdx.x] = tot;
      tot += c;
    }
  }
  __syncthreads();
  return tot;
}

// key of token t: pass 0 reads the ids, pass 1 the previous pass's keys
__device__ __forceinline__ int sort_key(const int64_t* ids, const int* kin, long long t, long long vstart, int vlocal) {
  if (kin) return kin[t];
  const long long l = ids[t] - vstart;
  return (l >= 0 && l < vlocal) ? (int)l : 0xFFFF;
}

__global__ __launch_bounds__(1024) void emb_digit_hist_k(const int64_t* __restrict__ ids, const int* __restrict__ kin,
                                                        long long vstart, int vlocal, int M, int shift,
                                                        int* __restrict__ table) {
  __shared__ int wc[16][256];
  const long long t = (long long)blockIdx.x * kSortChunk + threadIdx.x;
  const bool active = t < M;
  const int d = active ? (sort_key(ids, kin, t, vstart, vlocal) >> shift) & 255 : 0;
  const unsigned long long m = digit_match(d, active);
  const int tot = chunk_digit_prefix(wc, d, active, m);
  if (threadIdx.x < 256) table[threadIdx.x * gridDim.x + blockIdx.x] = tot;   // [digit][chunk]
}

__global__ __launch_bounds__(1024) void emb_digit_scatter_k(const int64_t* __restrict__ ids, const int* __restrict__ kin,
                                                           const int* __restrict__ vin, long long vstart, int vlocal,
                                                           int M, int shift, const int* __restrict__ table,
                                                           int* __restrict__ kout, int* __restrict__ vout,
                                                           int64_t* __restrict__ vout64) {
  __shared__ int wc[16][256];
  __shared__ int base[256];
  const int NC = gridDim.x, c = blockIdx.x;
  // the chunk's global offset of every digit: all chunks' counts of smaller digits, then this
  // digit's counts in earlier chunks (fixed-order sums: thread t < 256 owns digit t)
  __shared__ int dtot[256];
  if (threadIdx.x < 256) {
    int tot = 0, before = 0;
    for (int cc = 0; cc < NC; ++cc) {
      const int x = table[threadIdx.x * NC + cc];
      if (cc < c) before += x;
      tot += x;
    }
    dtot[threadIdx.x] = tot;
    base[threadIdx.x] = before;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int dd = 0; dd < 256; ++dd) {
      const int x = dtot[dd];
      dtot[dd] = run;
      run += x;
    }
  }
  __syncthreads();
  const long long t = (long long)c * kSortChunk + threadIdx.x;
  const bool active = t < M;
  const int key = active ? sort_key(ids, kin, t, vstart, vlocal) : 0;
  const int d = (key >> shift) & 255;
  const unsigned long long m = digit_match(d, active);
  chunk_digit_prefix(wc, d, active, m);
  if (active) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int pos = dtot[d] + base[d] + wc[w][d] + __popcll(m & lt);
    const int val = vin ? vin[t] : (int)t;
    kout[pos] = key;
    if (vout) vout[pos] = val;
    if (vout64) vout64[pos] = val;
  }
}

// seg[v] = first position of key >= v in the sorted keys, v = 0 .. vlocal
__global__ __launch_bounds__(256) void emb_seg_k(const int* __restrict__ keys, int M, int vlocal,
                                                int64_t* __restrict__ seg) {
  const int v = blockIdx.x * 256 + threadIdx.x;
  if (v > vlocal) return;
  int lo = 0, hi = M;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (keys[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  seg[v] = lo;
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

// Sorted / segmented form (embedding_bwd_seg_k): perm = the stable ascending order of the ids,
// seg[vlocal + 1] = each local vocab row's start in it.  D % 4 == 0.
extern "C" void dpfs_embedding_bwd_seg(int in_dtype, const void* dout, const int64_t* perm, const int64_t* seg, float* dw,
                                       int D, int vlocal, int accumulate, hipStream_t s) {
  const int grid = cap_grid2(vlocal, 4);
  if (in_dtype == kBF16)
    embedding_bwd_seg_k<bf16><<<grid, 256, 0, s>>>((const bf16*)dout, perm, seg, dw, D, vlocal, accumulate);
  else
    embedding_bwd_seg_k<float><<<grid, 256, 0, s>>>((const float*)dout, perm, seg, dw, D, vlocal, accumulate);
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

// ce_fused_k launcher: 1 = launched; 0 = not applicable (not bf16, V % 8, V > 8 * 512 * 13:
// the caller takes the two-pass path).  part: ce_fused_ws floats when dbias is wanted, else null.
static int ce_fused_grid(int M) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, c = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    cus = c;
  }
  return M < cus ? M : cus;
}

extern "C" long long dpfs_ce_fused_ws(int M, int V) { return (long long)ce_fused_grid(M) * V; }

extern "C" int dpfs_ce_fused(int dtype, void* logits, const int64_t* tgt, const float* gscale, float* stats,
                             float* dbias, float* part, int M, int V, long long vstart, int vvalid, hipStream_t s) {
  if (dtype != kBF16 || V % 8 != 0 || V <= 0) return 0;
  const int nv = (V / 8 + 511) / 512;
  if (nv > 13) return 0;   // (V <= 53248: past 13 slots the registers spill)
  if (M == 0) return 1;
  const int G = ce_fused_grid(M);
  float* pp = dbias ? part : nullptr;
#define CEF(N_) ce_fused_k<N_><<<G, 512, 0, s>>>((bf16*)logits, tgt, gscale, stats, pp, M, V, vstart, vvalid)
  switch (nv) {
    case 1: CEF(1); break;
    case 2: CEF(2); break;
    case 3: CEF(3); break;
    case 4: CEF(4); break;
    case 5: CEF(5); break;
    case 6: CEF(6); break;
    case 7: CEF(7); break;
    case 8: CEF(8); break;
    case 9: CEF(9); break;
    case 10: CEF(10); break;
    case 11: CEF(11); break;
    case 12: CEF(12); break;
    default: CEF(13); break;
  }
#undef CEF
  if (dbias) dpfs_colsum_rows_small(part, dbias, G, V, s);
  return 1;
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

// part: 2 * kCeBlocks floats of scratch
extern "C" int dpfs_ce_part_floats() { return 2 * kCeBlocks; }
extern "C" void dpfs_ce_finalize(const float* stats, const int64_t* tgt, long long ignore, float* lse, float* valid,
                                 float* acc, float* loss, float* part, int M, int nsh, int first, int last,
                                 hipStream_t s) {
  const int nb = std::max(1, std::min(kCeBlocks, (M + 255) / 256));
  ce_finalize_rows_k<<<nb, 256, 0, s>>>(stats, tgt, ignore, lse, valid, part, M, nsh);
  ce_finalize_sum_k<<<1, 64, 0, s>>>(part, nb, acc, loss, first, last);
}
extern "C" void dpfs_ce_valid_scale(const int64_t* tgt, long long ignore, float* gs, float* n_valid, float* part,
                                    int M, hipStream_t s) {
  const int nb = std::max(1, std::min(kCeBlocks, (M + 255) / 256));
  ce_valid_count_k<<<nb, 256, 0, s>>>(tgt, ignore, part, M);
  ce_valid_scale_k<<<nb, 256, 0, s>>>(tgt, ignore, part, gs, n_valid, M);
}

extern "C" void dpfs_ce_grad_scale(const float* valid, const void* gloss, int gloss_bf16, const float* n_valid,
                                   float* gs, int M, hipStream_t s) {
  if (M <= 0) return;
  const int nb = std::min(1024, (M + 255) / 256);
  if (gloss_bf16)
    ce_grad_scale_k<bf16><<<nb, 256, 0, s>>>(valid, (const bf16*)gloss, n_valid, gs, M);
  else
    ce_grad_scale_k<float><<<nb, 256, 0, s>>>(valid, (const float*)gloss, n_valid, gs, M);
}

// ws: 4 M + 256 * ceil(M / 1024) ints.  perm: int64 [M] (positions past seg[vlocal] hold the
// ids outside this shard), seg: int64 [vlocal + 1].
extern "C" long long dpfs_emb_sort_ws(int M) { return 4LL * M + 256LL * ((M + kSortChunk - 1) / kSortChunk); }
extern "C" void dpfs_emb_sort(const int64_t* ids, int M, long long vstart, int vlocal, int* ws, int64_t* perm,
                              int64_t* seg, hipStream_t s) {
  const int NC = (M + kSortChunk - 1) / kSortChunk;
  int *k1 = ws, *v1 = ws + M, *k2 = ws + 2LL * M, *table = ws + 4LL * M;
  if (M > 0) {
    emb_digit_hist_k<<<NC, 1024, 0, s>>>(ids, nullptr, vstart, vlocal, M, 0, table);
    emb_digit_scatter_k<<<NC, 1024, 0, s>>>(ids, nullptr, nullptr, vstart, vlocal, M, 0, table, k1, v1, nullptr);
    emb_digit_hist_k<<<NC, 1024, 0, s>>>(ids, k1, vstart, vlocal, M, 8, table);
    emb_digit_scatter_k<<<NC, 1024, 0, s>>>(ids, k1, v1, vstart, vlocal, M, 8, table, k2, nullptr, perm);
  }
  emb_seg_k<<<(vlocal + 1 + 255) / 256, 256, 0, s>>>(k2, M, vlocal, seg);
}
