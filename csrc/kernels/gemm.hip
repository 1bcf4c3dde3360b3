// bf16 MFMA GEMM for gfx950 (MI355X) — the three layouts of a tensor-parallel linear.
//
//   C[m][n] = sum_k A(m,k) B(k,n)       fp32 accumulate in MFMA accumulators
//
//   layout  A(m,k)            B(k,n)            use
//   NT      a[m*lda + k]      b[n*ldb + k]      forward   y  = x W^T (+bias)       (F.linear)
//   NN      a[m*lda + k]      b[k*ldb + n]      dgrad     dx = dy W
//   TN      a[k*lda + m]      b[k*ldb + n]      wgrad     dW = dy^T x   (fp32 out, split-K)
//
// Reference call sites: models/layers.py:49,93 (F.linear) and their autograd backward
// (SURVEY.md K8/K9).  Design (CDNA HIP guide §5):
//  * 128x128x64 block tile, 256 threads = 4 waves in 2x2, each wave 64x64 = 4x4 tiles of
//    v_mfma_f32_16x16x32_bf16 (16 accumulators x 4 regs);
//  * operands staged global -> registers (16-byte loads) -> LDS, double-buffered LDS with the
//    next tile's global loads issued BEFORE the current tile's MFMAs and written AFTER them
//    (async-STAGE split, T14), one barrier per K-step;
//  * K-contiguous operand tiles [rows][64] with an XOR chunk swizzle (chunk ^ row&7) read by
//    ds_read_b128; MN-contiguous tiles [64][128] (the transposed operands of dgrad/wgrad)
//    swizzled (chunk ^ 2h(row)) and read with the CDNA4 hardware-transpose read
//    ds_read_b64_tr_b16 (T10) — no transpose kernels, no scalar LDS traffic;
//  * bijective XCD-aware block remap (T1) with n fastest, so the blocks of one XCD share the
//    weight panel in their L2;
//  * edges: rows/cols masked on load (zero fill) and store; the contiguous dim of each
//    operand must be a multiple of 8 (16-byte vectors);
//  * split-K over blockIdx.y for the skinny-output wgrad: fp32 slabs + fixed-order reduction
//    (deterministic, no float atomics).
#include "common.h"

namespace dpfs {

constexpr int BM = 128, BN = 128, BKK = 64;
constexpr int kTileBytes = 128 * 64 * 2;  // 16 KiB per operand tile

// MN-major swizzle: rows read together by one ds_read_b64_tr_b16 half-wave are
// {b..b+3, b+8..b+11}; h() maps them to 8 distinct chunk pairs -> conflict-free.
__device__ __forceinline__ int mn_h(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

__device__ __forceinline__ int kmaj_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }
__device__ __forceinline__ int mnmaj_off(int row, int chunk) { return row * 256 + ((chunk ^ (mn_h(row) << 1)) << 4); }

template <bool KMAJ>
__device__ __forceinline__ void g2r(const bf16* __restrict__ P, int ld, int R, int K, int r0, int k0, u32x4 (&reg)[4]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = tid + 256 * i;
    int row, c;
    const bf16* src;
    bool ok;
    if (KMAJ) {
      row = q >> 3; c = q & 7;
      ok = (r0 + row < R) && (k0 + c * 8 < K);
      src = P + (long long)(r0 + row) * ld + k0 + c * 8;
    } else {
      row = q >> 4; c = q & 15;
      ok = (k0 + row < K) && (r0 + c * 8 < R);
      src = P + (long long)(k0 + row) * ld + r0 + c * 8;
    }
    u32x4 v = {0u, 0u, 0u, 0u};
    if (ok) v = *reinterpret_cast<const u32x4*>(src);
    reg[i] = v;
  }
}

template <bool KMAJ>
__device__ __forceinline__ void r2lds(char* lds, const u32x4 (&reg)[4]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = tid + 256 * i;
    const int off = KMAJ ? kmaj_off(q >> 3, q & 7) : mnmaj_off(q >> 4, q & 15);
    *reinterpret_cast<u32x4*>(lds + off) = reg[i];
  }
}

// Fragment of the 16x16x32 MFMA operand: lane l holds X[rb + (l&15)][kb + 8(l>>4) + j], j<8,
// where X is A (row = m) or B^T (row = n).
template <bool KMAJ>
__device__ __forceinline__ bf16x8 frag(const char* lds, int rb, int kb) {
  const int l = lane_id();
  if (KMAJ) {
    const int row = rb + (l & 15);
    const int chunk = (kb >> 3) + (l >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + kmaj_off(row, chunk));
  } else {
    const int i = l & 15, q = i >> 2, p = i & 3;
    const int col = rb + 4 * p;
    const int chunk = col >> 3;
    s16x4 lo, hi;
    {
      const int k = kb + 8 * (l >> 4) + q;
      lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(lds + mnmaj_off(k, chunk) + (p & 1) * 8));
    }
    {
      const int k = kb + 8 * (l >> 4) + 4 + q;
      hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(lds + mnmaj_off(k, chunk) + (p & 1) * 8));
    }
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// OUT: 0 = bf16 C (+ optional fp32 bias[n]); 1 = fp32 C slab (split-K partial or final).
template <bool AK, bool BKM, int OUT>
__global__ __launch_bounds__(256, 2) void gemm_k(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                 void* __restrict__ C, const float* __restrict__ bias, int M, int N,
                                                 int K, int lda, int ldb, int ldc, int k_per_split,
                                                 long long slab_stride) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * kTileBytes];
  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tm = wg / tiles_n, tn = wg % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.y * k_per_split;
  const int kend = min(K, kbeg + k_per_split);

  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int l = lane_id();

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  u32x4 ra[4], rb[4];
  const int nk = (kend - kbeg + BKK - 1) / BKK;
  if (nk > 0) {
    g2r<AK>(A, lda, M, kend, m0, kbeg, ra);
    g2r<BKM>(B, ldb, N, kend, n0, kbeg, rb);
    r2lds<AK>(smem, ra);
    r2lds<BKM>(smem + kTileBytes, rb);
  }
  __syncthreads();

  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    const char* la = smem + cur * 2 * kTileBytes;
    const char* lb = la + kTileBytes;
    const bool more = (t + 1) < nk;
    if (more) {
      const int k0 = kbeg + (t + 1) * BKK;
      g2r<AK>(A, lda, M, kend, m0, k0, ra);
      g2r<BKM>(B, ldb, N, kend, n0, k0, rb);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag<AK>(la, wm * 64 + i * 16, s * 32);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag<BKM>(lb, wn * 64 + j * 16, s * 32);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      char* na = smem + (cur ^ 1) * 2 * kTileBytes;
      r2lds<AK>(na, ra);
      r2lds<BKM>(na + kTileBytes, rb);
    }
    __syncthreads();
  }

  // Epilogue: C/D map of 16x16 MFMA: col = lane&15, row = 4*(lane>>4) + j.
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wn * 64 + j * 16 + (l & 15);
      if (col >= N) continue;
      float bv = 0.f;
      if (OUT == 0 && bias) bv = bias[col];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + i * 16 + 4 * (l >> 4) + r;
        if (row < M) {
          if (OUT == 0) {
            reinterpret_cast<bf16*>(C)[(long long)row * ldc + col] = (bf16)(acc[i][j][r] + bv);
          } else {
            reinterpret_cast<float*>(C)[blockIdx.y * slab_stride + (long long)row * ldc + col] = acc[i][j][r];
          }
        }
      }
    }
  }
}

// out[i] (+)= sum_s slab[s][i]  (fixed order), float4 vectorised; n % 4 == 0.
__global__ __launch_bounds__(256) void splitk_reduce_k(const float* __restrict__ slabs, float* __restrict__ out,
                                                       long long n, int S, int accumulate) {
  for (long long i = (blockIdx.x * (long long)blockDim.x + threadIdx.x) * 4; i < n;
       i += (long long)gridDim.x * blockDim.x * 4) {
    f32x4 s = accumulate ? *reinterpret_cast<const f32x4*>(out + i) : (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < S; ++k) s += *reinterpret_cast<const f32x4*>(slabs + k * n + i);
    *reinterpret_cast<f32x4*>(out + i) = s;
  }
}

}  // namespace dpfs

using namespace dpfs;

static int tiles_of(int M, int N) { return ((M + BM - 1) / BM) * ((N + BN - 1) / BN); }

// NT: C[M,N] bf16 = A[M,K] B[N,K]^T + bias
extern "C" void dpfs_gemm_nt(const void* A, const void* B, void* C, const float* bias, int M, int N, int K, int lda,
                             int ldb, int ldc, hipStream_t s) {
  dim3 grid(tiles_of(M, N), 1);
  gemm_k<true, true, 0><<<grid, 256, 0, s>>>((const bf16*)A, (const bf16*)B, C, bias, M, N, K, lda, ldb, ldc, K, 0);
}

// NN: C[M,N] bf16 = A[M,K] B[K,N]
extern "C" void dpfs_gemm_nn(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                             hipStream_t s) {
  dim3 grid(tiles_of(M, N), 1);
  gemm_k<true, false, 0><<<grid, 256, 0, s>>>((const bf16*)A, (const bf16*)B, C, nullptr, M, N, K, lda, ldb, ldc, K,
                                              0);
}

// How many K-splits the TN (wgrad) launch wants; the caller sizes the slab workspace as
// splits * M * N fp32 when splits > 1.
extern "C" int dpfs_gemm_tn_splits(int M, int N, int K) {
  const int tiles = tiles_of(M, N);
  int s = 1;
  while (tiles * s < 512 && (K / (s * 2)) >= 4 * BKK && s < 16) s *= 2;
  return s;
}

// TN: C[M,N] fp32 (+)= A[K,M]^T B[K,N].  ws: splits*M*N floats when splits > 1.
extern "C" void dpfs_gemm_tn(const void* A, const void* B, float* C, float* ws, int M, int N, int K, int lda, int ldb,
                             int accumulate, hipStream_t s) {
  const int S = dpfs_gemm_tn_splits(M, N, K);
  int kps = (K + S - 1) / S;
  kps = ((kps + BKK - 1) / BKK) * BKK;
  const long long n = (long long)M * N;
  if (S == 1 && !accumulate) {
    gemm_k<false, false, 1><<<dim3(tiles_of(M, N), 1), 256, 0, s>>>((const bf16*)A, (const bf16*)B, C, nullptr, M, N,
                                                                   K, lda, ldb, N, K, 0);
    return;
  }
  gemm_k<false, false, 1><<<dim3(tiles_of(M, N), S), 256, 0, s>>>((const bf16*)A, (const bf16*)B, ws, nullptr, M, N,
                                                                 K, lda, ldb, N, kps, n);
  long long g = (n / 4 + 255) / 256;
  if (g > 4096) g = 4096;
  splitk_reduce_k<<<(int)g, 256, 0, s>>>(ws, C, n, S, accumulate);
}
