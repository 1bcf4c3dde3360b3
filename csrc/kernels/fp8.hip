// Per-tensor fp8 quantisation for the optional fp8 GEMM path (gfx950: OCP e4m3fn / e5m2,
// the formats of v_cvt_pk_fp8_f32 / v_cvt_pk_bf8_f32 and of hipBLASLt's fp8 MFMA GEMMs).
//
// "Current" scaling: amax over the whole tensor, scale = FMAX / amax, q = sat(x * scale),
// and the GEMM gets inv = 1 / scale (torch._scaled_mm's scale_a / scale_b).  Two kernels, no
// host round trip: amax_k writes per-workgroup maxima, cast_k reduces them and casts, so the
// whole quantisation is stream-ordered and graph-capturable.  The fp32 scale arithmetic matches the
// PyTorch oracle (ops/fp8.py) operation for operation, so the fp8 bytes are identical.
#include "common.h"
#include <hip/hip_fp8.h>

namespace dpfs {

// Per-workgroup maxima into part[gridDim.x] (no atomics: 2048 same-address atomic maxima cost
// ~20 us, more than the pass itself); the cast kernel reduces the partials.
__global__ __launch_bounds__(256) void fp8_amax_k(const bf16* __restrict__ x, long long nvec,
                                                  float* __restrict__ part) {
  float m = 0.f;
#pragma unroll 4
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nvec; i += (long long)gridDim.x * blockDim.x) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + 8 * i);
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf((float)v[j]));
  }
  m = wave_max(m);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

template <int FMT>   // 0 = e4m3 (OCP e4m3fn), 1 = e5m2
__global__ __launch_bounds__(256) void fp8_cast_k(const bf16* __restrict__ x, long long nvec,
                                                  const float* __restrict__ part, int nparts,
                                                  unsigned long long* __restrict__ out, float* __restrict__ inv) {
  constexpr float FMAX = FMT == 0 ? 448.f : 57344.f;
  constexpr __hip_fp8_interpretation_t I = FMT == 0 ? __HIP_E4M3 : __HIP_E5M2;
  // amax = max of the partials (every workgroup reduces the same <= 512 values: a few KB of L2)
  float pm = 0.f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) pm = fmaxf(pm, part[i]);
  pm = wave_max(pm);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = pm;
  __syncthreads();
  const float amax = fmaxf(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])), 1e-12f);
  const float scale = FMAX / amax;
  if (blockIdx.x == 0 && threadIdx.x == 0) *inv = 1.f / scale;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nvec; i += (long long)gridDim.x * blockDim.x) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + 8 * i);
    unsigned long long r = 0;
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const float2 f = make_float2((float)v[j] * scale, (float)v[j + 1] * scale);
      const __hip_fp8x2_storage_t p = __hip_cvt_float2_to_fp8x2(f, __HIP_SATFINITE, I);
      r |= (unsigned long long)(unsigned short)p << (8 * j);
    }
    out[i] = r;
  }
}

}  // namespace dpfs

using namespace dpfs;

// x: n bf16 (n % 8 == 0, 16-byte aligned); out: n fp8 bytes (8-byte aligned); inv: 1 fp32;
// work: >= 512 fp32 of scratch (the per-workgroup maxima).
extern "C" int dpfs_fp8_work_floats() { return 512; }

extern "C" void dpfs_fp8_quant(const void* x, long long n, int fmt, void* out, float* inv, float* work,
                               hipStream_t s) {
  const long long nvec = n / 8;
  long long ga = (nvec + 255) / 256;
  if (ga > 512) ga = 512;
  if (ga < 1) ga = 1;
  long long gc = (nvec + 255) / 256;
  if (gc > 2048) gc = 2048;
  if (gc < 1) gc = 1;
  fp8_amax_k<<<(int)ga, 256, 0, s>>>((const bf16*)x, nvec, work);
  if (fmt == 0)
    fp8_cast_k<0><<<(int)gc, 256, 0, s>>>((const bf16*)x, nvec, work, (int)ga, (unsigned long long*)out, inv);
  else
    fp8_cast_k<1><<<(int)gc, 256, 0, s>>>((const bf16*)x, nvec, work, (int)ga, (unsigned long long*)out, inv);
}
