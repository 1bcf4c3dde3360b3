// Store-shape probe: how fast does a wave write a 128 x 128 bf16 tile (32 KiB, 32 buffer
// stores of 16 bytes per lane) depending on how many rows one store instruction spans?
//   shape 16: 16 rows x 64 B per instruction (the GEMM epilogue's current form)
//   shape  8:  8 rows x 128 B (whole 128-byte lines)
//   shape  4:  4 rows x 256 B
// Every wave writes its own tile of a (rows x cols) bf16 matrix; the kernel time over the
// total bytes gives the store rate.  Build: hipcc --offload-arch=gfx950 -O3 tools/store_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int RPI>   // rows per instruction
__global__ __launch_bounds__(256) void store_tiles(unsigned short* C, int rows, int cols, int tiles_n) {
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + wave;               // wave tile index
  const int tm = t / tiles_n, tn = t % tiles_n;
  const int r0 = tm * 128, c0 = tn * 128;
  if (r0 >= rows) return;
  constexpr int LPR = 64 / RPI;                      // lanes per row, 16 B each
  const int lr = l / LPR, lc = l % LPR;
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
      C, (short)0, (int)((long long)rows * cols * 2 > 0x7fffffff ? 0x7fffffff : (long long)rows * cols * 2), 0x00020000);
  const u32x4 v = {(unsigned)l, (unsigned)t, 7u, 9u};
  // 32 instructions cover 128 rows x 256 B: each instruction RPI rows x (LPR x 16 B)
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    // instruction i: row block (i * RPI) % 128, column chunk (i * RPI) / 128
    const int rb = (i * RPI) % 128, cb = (i * RPI) / 128;
    const int row = r0 + rb + lr, col = c0 + cb * (LPR * 8) + lc * 8;
    const unsigned off = (unsigned)(((long long)row * cols + col) * 2);
    __builtin_amdgcn_raw_buffer_store_b128(v, rc, off, 0, 0);
  }
}

template <int RPI>
float run(unsigned short* C, int rows, int cols, int reps) {
  const int tiles_n = cols / 128, tiles = rows / 128 * tiles_n;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  store_tiles<RPI><<<tiles / 4, 256>>>(C, rows, cols, tiles_n);
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r) store_tiles<RPI><<<tiles / 4, 256>>>(C, rows, cols, tiles_n);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main(int argc, char** argv) {
  const int rows = argc > 1 ? atoi(argv[1]) : 32768, cols = argc > 2 ? atoi(argv[2]) : 4096;
  unsigned short* C = nullptr;
  if (hipMalloc(&C, (size_t)rows * cols * 2) != hipSuccess) return 1;
  const double bytes = (double)rows * cols * 2;
  for (int round = 0; round < 3; ++round) {
    const float t16 = run<16>(C, rows, cols, 20), t8 = run<8>(C, rows, cols, 20), t4 = run<4>(C, rows, cols, 20);
    printf("rows %d cols %d: 16 rows x 64 B %.4f ms (%.2f TB/s)   8 rows x 128 B %.4f ms (%.2f TB/s)   "
           "4 rows x 256 B %.4f ms (%.2f TB/s)\n",
           rows, cols, t16, bytes / t16 / 1e9, t8, bytes / t8 / 1e9, t4, bytes / t4 / 1e9);
  }
  hipFree(C);
  return 0;
}
