// Probe: does hipBLASLt have a faster algorithm than its heuristic's first choice (the one
// torch.nn.functional.linear / torch.matmul run) on the GPT-2-small step's plain GEMMs?
// For each shape: ask the heuristic for up to 64 algorithms, time each (best of 3 x 10 reps),
// print heuristic #0 vs the fastest.  Standalone (no torch): build with
//   hipcc --offload-arch=gfx950 -O2 tools/blaslt_probe.cpp -o build/blaslt_probe -L<lib> -lhipblaslt
// against /opt/rocm/lib or torch/lib to compare the two library builds.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                           \
  do {                                                                                  \
    auto _e = (x);                                                                      \
    if ((int)_e != 0) {                                                                 \
      std::fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, (int)_e);        \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

__global__ void fill_k(__hip_bfloat16* p, long long n, unsigned seed) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    p[i] = __float2bfloat16(((float)(h & 0xffff) / 65536.f - 0.5f) * 0.1f);
  }
}

struct Shape {
  const char* name;
  int layout;  // 0 = NT: y[M,N] = x[M,K] w[N,K]^T ; 1 = NN: y[M,N] = a[M,K] b[K,N];
               // 2 = TN: fp32 y[M,N] += a[K,M]^T b[K,N] (weight gradient, accumulate)
  int M, N, K;
  bool bias;
};

int main(int argc, char** argv) {
  const int maxalgo = argc > 1 ? std::atoi(argv[1]) : 64;
  std::vector<Shape> shapes = {
      {"qkv fwd", 0, 32768, 2304, 768, true},      {"wo fwd", 0, 32768, 768, 768, true},
      {"gate|up fwd", 0, 32768, 4096, 768, true},  {"down fwd", 0, 32768, 768, 2048, true},
      {"lm_head fwd", 0, 32768, 50304, 768, true}, {"qkv dgrad", 1, 32768, 768, 2304, false},
      {"wo dgrad", 1, 32768, 768, 768, false},     {"gate|up dgrad", 1, 32768, 768, 4096, false},
      {"down dgrad", 1, 32768, 2048, 768, false},  {"lm_head dgrad", 1, 32768, 768, 50304, false},
      {"qkv wgrad", 2, 2304, 768, 32768, false},   {"wo wgrad", 2, 768, 768, 32768, false},
      {"gate|up wgrad", 2, 4096, 768, 32768, false}, {"down wgrad", 2, 768, 2048, 32768, false},
      {"lm_head wgrad", 2, 50304, 768, 32768, false},
  };
  hipblasLtHandle_t h;
  CK(hipblasLtCreate(&h));
  int ver = 0;
  hipblasLtGetVersion(h, &ver);
  std::printf("hipBLASLt version %d\n", ver);
  const size_t ws_bytes = 128ull << 20;
  void* ws;
  CK(hipMalloc(&ws, ws_bytes));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Shape& sh : shapes) {
    const long long na = (long long)sh.M * sh.K, nb = (long long)sh.N * sh.K, nd = (long long)sh.M * sh.N;
    const bool tn = sh.layout == 2;
    __hip_bfloat16 *x, *w;
    void* y;
    float* bias;
    CK(hipMalloc(&x, na * 2));
    CK(hipMalloc(&w, nb * 2));
    CK(hipMalloc(&y, nd * (tn ? 4 : 2)));
    CK(hipMemsetAsync(y, 0, nd * (tn ? 4 : 2), s));
    CK(hipMalloc(&bias, sh.N * 4));
    fill_k<<<1024, 256, 0, s>>>(x, na, 1);
    fill_k<<<1024, 256, 0, s>>>(w, nb, 2);
    CK(hipMemsetAsync(bias, 0, sh.N * 4, s));
    // column-major view: D^T[N, M] = op(A) op(B), A = w, B = x
    hipblasLtMatmulDesc_t desc;
    CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    // TN: D^T[N, M] = b^T[N, K] a[K, M]: A = b (col-major [N, K], ld N, no trans),
    //     B = a (col-major [M, K] ld M -> trans)
    hipblasOperation_t ta = sh.layout == 0 ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = tn ? HIPBLAS_OP_T : HIPBLAS_OP_N;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
    if (sh.bias) {
      hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
      hipDataType bt = HIP_R_32F;
      CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)));
      CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
      CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
    }
    hipblasLtMatrixLayout_t la, lb, ld;
    if (sh.layout == 0)
      CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, sh.K, sh.N, sh.K));  // w [N,K] row-major
    else
      CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, sh.N, sh.K, sh.N));  // b [K,N] row-major
    if (tn)
      CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, sh.M, sh.K, sh.M));  // a [K,M] row-major
    else
      CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, sh.K, sh.M, sh.K));  // x [M,K] row-major
    CK(hipblasLtMatrixLayoutCreate(&ld, tn ? HIP_R_32F : HIP_R_16BF, sh.N, sh.M, sh.N));  // y [M,N] row-major
    hipblasLtMatmulPreference_t pref;
    CK(hipblasLtMatmulPreferenceCreate(&pref));
    uint64_t wsb = ws_bytes;
    CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
    std::vector<hipblasLtMatmulHeuristicResult_t> res(maxalgo);
    int got = 0;
    CK(hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, ld, ld, pref, maxalgo, res.data(), &got));
    const float alpha = 1.f, beta = tn ? 1.f : 0.f;
    int nok = 0;
    std::vector<double> all;
    double t0 = -1, best = 1e30;
    int besti = -1;
    for (int i = 0; i < got; ++i) {
      if (res[i].state != HIPBLAS_STATUS_SUCCESS || res[i].workspaceSize > ws_bytes) continue;
      auto run = [&]() {
        return hipblasLtMatmul(h, desc, &alpha, w, la, x, lb, &beta, y, ld, y, ld, &res[i].algo, ws, ws_bytes, s);
      };
      if (run() != HIPBLAS_STATUS_SUCCESS) continue;
      double t = 1e30;
      for (int r = 0; r < 3; ++r) {
        CK(hipEventRecord(e0, s));
        for (int k = 0; k < 10; ++k) run();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t = std::min(t, (double)ms / 10);
      }
      if (i == 0) t0 = t;
      ++nok;
      all.push_back(t);
      if (t < best) {
        best = t;
        besti = i;
      }
    }
    const double fl = 2.0 * sh.M * sh.N * sh.K;
    std::sort(all.begin(), all.end());
    std::printf("  ran %d algos, median %.4f ms\n", nok, all.empty() ? 0.0 : all[all.size() / 2]);
    std::printf("%-14s %s M=%d N=%d K=%d  algos=%d  heuristic#0 %.4f ms (%.0f TF/s)  best #%d %.4f ms (%.0f TF/s)  gain %.1f%%\n",
                sh.name, sh.layout == 0 ? "NT" : (tn ? "TN" : "NN"), sh.M, sh.N, sh.K, got, t0, fl / t0 / 1e9, besti, best,
                fl / best / 1e9, t0 > 0 ? 100.0 * (t0 - best) / t0 : 0.0);
    std::fflush(stdout);
    hipblasLtMatmulPreferenceDestroy(pref);
    hipblasLtMatrixLayoutDestroy(la);
    hipblasLtMatrixLayoutDestroy(lb);
    hipblasLtMatrixLayoutDestroy(ld);
    hipblasLtMatmulDescDestroy(desc);
    CK(hipFree(x));
    CK(hipFree(w));
    CK(hipFree(y));
    CK(hipFree(bias));
  }
  return 0;
}
