// Shared device helpers for the gfx950 (MI355X, CDNA4) kernels.
//
// Conventions used by every kernel in this directory:
//  * wave64: every reduction is a 64-lane butterfly (__shfl_xor over 64 lanes);
//  * 16-byte vector memory access per lane (8 x bf16 or 4 x fp32), Guideline 13 of the
//    CDNA HIP guide: scalar bf16 loads cost 2-2.5x;
//  * fp32 math / accumulation, bf16 storage; bf16 rounding via the native conversion
//    (hipcc -O3 emits v_cvt_pk_bf16_f32, which keeps NaNs NaN);
//  * launchers are extern "C", take raw device pointers + hipStream_t and never
//    allocate or synchronise (graph-capturable).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// Device-side bounds asserts of the DPFS_KERNEL_ASSERT=1 build (python tools/build_ext.py
// --kernel-assert -> _C_kassert*.so, loaded when DPFS_KERNEL_ASSERT=1 is set at run time):
// a failed check prints the file, line, condition and the offending values, then traps the
// wave (the launch fails with a device exception at the next synchronisation).  In the
// default build the macro is empty, so the hot kernels carry no extra instruction.
#if defined(DPFS_KERNEL_ASSERT) && DPFS_KERNEL_ASSERT
#define KASSERT(cond, fmt, ...)                                                             \
  do {                                                                                          \
    if (!(cond)) {                                                                              \
      printf("[dpfs kernel assert] %s:%d: %s (block %d, thread %d): " fmt "\n", __FILE__, __LINE__, \
             #cond, (int)blockIdx.x, (int)threadIdx.x, ##__VA_ARGS__);                          \
      __builtin_trap();                                                                         \
    }                                                                                           \
  } while (0)
#else
#define KASSERT(cond, fmt, ...) \
  do {                               \
  } while (0)
#endif

namespace dpfs {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

enum DType : int { kF32 = 0, kBF16 = 1 };

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }

// 16-byte vector of T: 8 bf16 or 4 fp32.
template <typename T> struct Vec;
template <> struct Vec<bf16> {
  static constexpr int N = 8;
  typedef bf16x8 type;
};
template <> struct Vec<float> {
  static constexpr int N = 4;
  typedef f32x4 type;
};

template <typename T>
__device__ __forceinline__ void load_vec(const T* p, float (&out)[Vec<T>::N]) {
  typename Vec<T>::type v = *reinterpret_cast<const typename Vec<T>::type*>(p);
#pragma unroll
  for (int i = 0; i < Vec<T>::N; ++i) out[i] = to_f(v[i]);
}

template <typename T>
__device__ __forceinline__ void store_vec(T* p, const float (&in)[Vec<T>::N]) {
  typename Vec<T>::type v;
#pragma unroll
  for (int i = 0; i < Vec<T>::N; ++i) v[i] = from_f<T>(in[i]);
  *reinterpret_cast<typename Vec<T>::type*>(p) = v;
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

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Bijective XCD-aware remap of a linear workgroup id (MI355X: 8 XCDs, dispatch deals
// blocks round-robin over XCDs).  Consecutive remapped ids land on the same XCD, so tiles
// that share operand panels share an L2.  Valid for any nwg (the q/r form).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int NX = 8;
  int xcd = orig % NX;
  int q = nwg / NX, r = nwg % NX;
  int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / NX;
}

// ---- LDS-DMA (buffer_load ... lds) helpers shared by the GEMM and attention kernels.
// A per-lane source offset past the descriptor's num_records returns zeros.
constexpr unsigned kOOB = 0xFFFFFFF0u;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds_wave_base, unsigned off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, off, 0,
                                           0, 0);
}

template <int N_>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N_ >= 0 && N_ < 64, "vmcnt range");
  // gfx9 s_waitcnt: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14]
  __builtin_amdgcn_s_waitcnt((N_ & 15) | (7 << 4) | (15 << 8) | ((N_ >> 4) << 14));
}

// Sums over the 32 lanes of each wave half of N per-lane values (N a multiple of 32), as a
// transpose reduction: at each halving step (partner lane l ^ m, m = 16, 8, 4, 2, 1) a lane
// keeps the half of its values that its lane bit m selects and adds the partner's copy of that
// half -- N - N/32 lane exchanges for the whole reduction instead of 5 N for a butterfly per
// value.  m = 16 is v_permlane16_swap (VALU; called with (lower half, upper half) the swap hands
// an even-row lane the partner's lower half and an odd-row lane the partner's upper half, so no
// select); m = 8 .. 1 are ds_swizzle xor exchanges of the half the partner keeps.  On return lane
// r32 holds in w[j] the sum of value r32 (N / 32) + j, j < N / 32 (the rest of w is scratch).
template <int N>
__device__ __forceinline__ void lane32_sums(float (&w)[N], int r32) {
  static_assert(N % 32 == 0, "lane32_sums: N must be a multiple of 32");
#pragma unroll
  for (int k = 0; k < N / 2; ++k) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(w[k]), __float_as_uint(w[k + N / 2]), false, false);
    w[k] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
#define LANE32_STEP(M_, n_)                                                                        \
  {                                                                                                \
    const bool hi = r32 & (M_);                                                                    \
    _Pragma("unroll") for (int k = 0; k < (n_) / 2; ++k) {                                         \
      const float send = hi ? w[k] : w[k + (n_) / 2], keep = hi ? w[k + (n_) / 2] : w[k];          \
      w[k] = keep + __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(send), 0x1F | ((M_) << 10))); \
    }                                                                                              \
  }
  LANE32_STEP(8, N / 2)
  LANE32_STEP(4, N / 4)
  LANE32_STEP(2, N / 8)
  LANE32_STEP(1, N / 16)
#undef LANE32_STEP
}

}  // namespace dpfs

#define LAUNCH_CHECK() (void)hipGetLastError()
