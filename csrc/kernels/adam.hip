// Multi-tensor fused Adam for gfx950 (replaces torch.optim.Adam's foreach kernels,
// reference train.py:83,108).
//
// ONE launch updates every parameter of the model: a device-resident descriptor table
// (one entry per tensor: fp32 master, fp32 grad, exp_avg, exp_avg_sq, optional bf16 shadow)
// and a chunk table (tensor, chunk) built once by the host.  Each 256-thread block streams
// one 16K-element chunk with 16-byte accesses, updates the master weights in fp32 and
// writes the bf16 compute shadow in the same pass, so the forward GEMMs never run a cast
// kernel.  Semantics = torch.optim.Adam (L2 weight decay added to the gradient; bias
// correction with the step count).  Optional device-side grad scale (clip coefficient)
// keeps gradient clipping free of host syncs.
#include "common.h"

namespace dpfs {

struct AdamTensor {
  float* p;
  const float* g;
  float* m;
  float* v;
  bf16* shadow;
  long long n;
};

constexpr int kAdamChunk = 16384;

__global__ __launch_bounds__(256) void adam_k(const AdamTensor* __restrict__ ts, const int* __restrict__ chunks,
                                              float lr, float b1, float b2, float eps, float wd, float bc1,
                                              float bc2_sqrt, float gscale, const float* __restrict__ dscale) {
  const int t = chunks[blockIdx.x * 2];
  const long long c0 = (long long)chunks[blockIdx.x * 2 + 1] * kAdamChunk;
  const AdamTensor T = ts[t];
  const long long c1 = min(T.n, c0 + kAdamChunk);
  const float scale = gscale * (dscale ? *dscale : 1.f);
  const float step = lr / bc1;
  const bool vec = ((T.n & 3) == 0);
  if (vec) {
    for (long long i = c0 + threadIdx.x * 4; i < c1; i += blockDim.x * 4) {
      f32x4 p = *reinterpret_cast<f32x4*>(T.p + i);
      f32x4 g = *reinterpret_cast<const f32x4*>(T.g + i);
      f32x4 m = *reinterpret_cast<f32x4*>(T.m + i);
      f32x4 v = *reinterpret_cast<f32x4*>(T.v + i);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float gg = g[j] * scale + wd * p[j];
        m[j] = b1 * m[j] + (1.f - b1) * gg;
        v[j] = b2 * v[j] + (1.f - b2) * gg * gg;
        p[j] -= step * m[j] / (sqrtf(v[j]) / bc2_sqrt + eps);
      }
      *reinterpret_cast<f32x4*>(T.p + i) = p;
      *reinterpret_cast<f32x4*>(T.m + i) = m;
      *reinterpret_cast<f32x4*>(T.v + i) = v;
      if (T.shadow) {
        bf16x4 s = {(bf16)p[0], (bf16)p[1], (bf16)p[2], (bf16)p[3]};
        *reinterpret_cast<bf16x4*>(T.shadow + i) = s;
      }
    }
  } else {
    for (long long i = c0 + threadIdx.x; i < c1; i += blockDim.x) {
      float p = T.p[i];
      float gg = T.g[i] * scale + wd * p;
      float m = b1 * T.m[i] + (1.f - b1) * gg;
      float v = b2 * T.v[i] + (1.f - b2) * gg * gg;
      p -= step * m / (sqrtf(v) / bc2_sqrt + eps);
      T.p[i] = p;
      T.m[i] = m;
      T.v[i] = v;
      if (T.shadow) T.shadow[i] = (bf16)p;
    }
  }
}

// Sum of squares of all grads (for global-norm clipping), per-chunk partials (fixed order).
__global__ __launch_bounds__(256) void sumsq_k(const AdamTensor* __restrict__ ts, const int* __restrict__ chunks,
                                               float* __restrict__ partial) {
  const int t = chunks[blockIdx.x * 2];
  const long long c0 = (long long)chunks[blockIdx.x * 2 + 1] * kAdamChunk;
  const AdamTensor T = ts[t];
  const long long c1 = min(T.n, c0 + kAdamChunk);
  float s = 0.f;
  for (long long i = c0 + threadIdx.x; i < c1; i += blockDim.x) s += T.g[i] * T.g[i];
  s = wave_sum(s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

}  // namespace dpfs

using namespace dpfs;

// Gradient pointers of the descriptor table, rewritten in place from kernel arguments (up to
// kPatch per launch): the training engine hands back fresh gradient tensors every step, and
// an H2D copy of a rebuilt table would stall the stream on a host round trip.
namespace dpfs {
constexpr int kPatch = 256;
struct GradPtrs {
  long long v[kPatch];
};
__global__ __launch_bounds__(256) void adam_patch_grads_k(AdamTensor* __restrict__ ts, GradPtrs p, int i0, int n) {
  const int i = threadIdx.x;
  if (i < n) ts[i0 + i].g = reinterpret_cast<const float*>(p.v[i]);
}
}  // namespace dpfs

extern "C" void dpfs_adam_patch_grads(void* desc, const long long* ptrs, int n, hipStream_t s) {
  for (int i0 = 0; i0 < n; i0 += kPatch) {
    GradPtrs p;
    const int m = n - i0 < kPatch ? n - i0 : kPatch;
    for (int i = 0; i < m; ++i) p.v[i] = ptrs[i0 + i];
    adam_patch_grads_k<<<1, 256, 0, s>>>(reinterpret_cast<AdamTensor*>(desc), p, i0, m);
  }
}

extern "C" int dpfs_adam_chunk() { return kAdamChunk; }
extern "C" int dpfs_adam_desc_bytes() { return (int)sizeof(AdamTensor); }

extern "C" void dpfs_adam_step(const void* desc, const int* chunks, int n_chunks, float lr, float b1, float b2,
                               float eps, float wd, float bc1, float bc2_sqrt, float gscale, const float* dscale,
                               hipStream_t s) {
  if (n_chunks == 0) return;
  adam_k<<<n_chunks, 256, 0, s>>>((const AdamTensor*)desc, chunks, lr, b1, b2, eps, wd, bc1, bc2_sqrt, gscale,
                                  dscale);
}

extern "C" void dpfs_grad_sumsq(const void* desc, const int* chunks, int n_chunks, float* partial, hipStream_t s) {
  if (n_chunks == 0) return;
  sumsq_k<<<n_chunks, 256, 0, s>>>((const AdamTensor*)desc, chunks, partial);
}
