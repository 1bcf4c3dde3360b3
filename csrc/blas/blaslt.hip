// hipBLASLt driven directly (the library PyTorch itself loads: torch/lib/libhipblaslt.so, same
// instance), for the plain GEMMs where its heuristic's FIRST algorithm -- the one
// torch.nn.functional.linear / torch.matmul / mm(out_dtype=fp32) run -- is not its fastest.
//
// tools/blaslt_probe.cpp / tools/lt_probe.py on MI355X (GPT-2 small step shapes, 64 heuristic
// algorithms each): for several projections an algorithm further down the list beats heuristic
// #0 by 4-17 % (profiles/r2_blaslt_probe.txt).  The plan (descriptors + the heuristic's
// algorithm list) is built once per shape; which algorithm runs is chosen by
// ops/gemm_select.py, by timing on the live operands against our kernels and torch's path.
//
// Row-major PyTorch tensors are handed to the column-major library as their transposes:
//   0 NT  y[M,N]  = x[M,K] w[N,K]^T (+ bias[N] fp32)  ->  D^T[N,M] = op_T(w) x^T
//   1 NN  y[M,N]  = a[M,K] b[K,N]                      ->  D^T[N,M] = b^T a^T
//   2 TN  y[M,N] (+)= a[K,M]^T b[K,N], y fp32          ->  D^T[N,M] = b^T op_T(a^T)
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

namespace {

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, ld = nullptr;
  std::vector<hipblasLtMatmulHeuristicResult_t> algos;
};

using Key = std::tuple<int, long long, long long, long long, int, int>;  // layout, M, N, K, bias, device

std::mutex g_mu;
std::map<Key, Plan*> g_plans;
hipblasLtHandle_t g_handle[16] = {nullptr};
char g_err[256] = "";

constexpr int kMaxAlgos = 64;
constexpr unsigned long long kMaxWorkspace = 128ull << 20;

bool ok(hipblasStatus_t s, const char* what) {
  if (s == HIPBLAS_STATUS_SUCCESS) return true;
  std::snprintf(g_err, sizeof(g_err), "%s failed: hipblasStatus %d", what, (int)s);
  return false;
}

hipblasLtHandle_t handle_for(int dev) {
  if (dev < 0 || dev >= 16) return nullptr;
  if (!g_handle[dev] && !ok(hipblasLtCreate(&g_handle[dev]), "hipblasLtCreate")) return nullptr;
  return g_handle[dev];
}

Plan* build(int layout, long long M, long long N, long long K, int bias, hipblasLtHandle_t h) {
  Plan* p = new Plan();
  bool good = ok(hipblasLtMatmulDescCreate(&p->desc, HIPBLAS_COMPUTE_32F, HIP_R_32F), "MatmulDescCreate");
  const hipblasOperation_t ta = layout == 0 ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  const hipblasOperation_t tb = layout == 2 ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  good = good && ok(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)), "TRANSA");
  good = good && ok(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)), "TRANSB");
  if (good && bias) {
    const hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
    const hipDataType bt = HIP_R_32F;
    good = ok(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)), "EPILOGUE") &&
           ok(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)),
              "BIAS_DATA_TYPE");
  }
  // A: w [N,K] (NT, transposed) or b [K,N] (NN, TN);  B: x [M,K] (NT, NN) or a [K,M] (TN, transposed)
  if (good) {
    good = layout == 0 ? ok(hipblasLtMatrixLayoutCreate(&p->la, HIP_R_16BF, K, N, K), "layout A")
                       : ok(hipblasLtMatrixLayoutCreate(&p->la, HIP_R_16BF, N, K, N), "layout A");
  }
  if (good) {
    good = layout == 2 ? ok(hipblasLtMatrixLayoutCreate(&p->lb, HIP_R_16BF, M, K, M), "layout B")
                       : ok(hipblasLtMatrixLayoutCreate(&p->lb, HIP_R_16BF, K, M, K), "layout B");
  }
  if (good)
    good = ok(hipblasLtMatrixLayoutCreate(&p->ld, layout == 2 ? HIP_R_32F : HIP_R_16BF, N, M, N), "layout D");
  if (good) {
    hipblasLtMatmulPreference_t pref = nullptr;
    good = ok(hipblasLtMatmulPreferenceCreate(&pref), "PreferenceCreate");
    const unsigned long long ws = kMaxWorkspace;
    good = good && ok(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws,
                                                            sizeof(ws)),
                      "PREF_MAX_WORKSPACE_BYTES");
    std::vector<hipblasLtMatmulHeuristicResult_t> res(kMaxAlgos);
    int got = 0;
    good = good && ok(hipblasLtMatmulAlgoGetHeuristic(h, p->desc, p->la, p->lb, p->ld, p->ld, pref, kMaxAlgos,
                                                      res.data(), &got),
                      "AlgoGetHeuristic");
    if (pref) hipblasLtMatmulPreferenceDestroy(pref);
    for (int i = 0; good && i < got; ++i)
      if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize <= kMaxWorkspace) p->algos.push_back(res[i]);
  }
  return p;  // an unusable plan keeps algos empty (the caller then never selects it)
}

Plan* plan_for(int layout, long long M, long long N, long long K, int bias, hipblasLtHandle_t* hout = nullptr) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  const Key key{layout, M, N, K, bias, dev};
  std::lock_guard<std::mutex> g(g_mu);
  hipblasLtHandle_t h = handle_for(dev);
  if (!h) return nullptr;
  if (hout) *hout = h;
  auto it = g_plans.find(key);
  if (it != g_plans.end()) return it->second;
  Plan* p = build(layout, M, N, K, bias, h);
  g_plans[key] = p;
  return p;
}

}  // namespace

extern "C" const char* dpfs_lt_last_error() { return g_err; }

// Number of usable algorithms for this problem (0: hipBLASLt has none / plan failed).
extern "C" int dpfs_lt_algos(int layout, long long M, long long N, long long K, int bias) {
  if (layout < 0 || layout > 2 || M <= 0 || N <= 0 || K <= 0 || (bias && layout != 0)) return 0;
  Plan* p = plan_for(layout, M, N, K, bias);
  return p ? (int)p->algos.size() : 0;
}

// Workspace bytes to hand algorithm i: the preference limit, not the heuristic's reported
// minimum -- the split-K / stream-K kernels size their split count to the workspace they are
// given at run time (with the minimum, the K = 32768 weight-gradient GEMMs ran ~1.6x slower).
extern "C" long long dpfs_lt_workspace(int layout, long long M, long long N, long long K, int bias, int i) {
  Plan* p = plan_for(layout, M, N, K, bias);
  if (!p || i < 0 || i >= (int)p->algos.size()) return -1;
  const long long need = (long long)p->algos[i].workspaceSize;
  return need > (long long)kMaxWorkspace ? need : (long long)kMaxWorkspace;
}

// Run algorithm i.  op_a / op_b are the row-major operands in the order of the layout comment
// (NT: x, w;  NN: a, b;  TN: a, b); d is y.  beta 0 overwrites, 1 accumulates (TN).
// Returns 0 on success, else a hipblasStatus (message in dpfs_lt_last_error()).
extern "C" int dpfs_lt_run(int layout, long long M, long long N, long long K, const float* bias, int i,
                           const void* op_a, const void* op_b, void* d, float beta, void* ws, long long ws_bytes,
                           hipStream_t s) {
  hipblasLtHandle_t h = nullptr;
  Plan* p = plan_for(layout, M, N, K, bias != nullptr, &h);
  if (!p || i < 0 || i >= (int)p->algos.size()) {
    std::snprintf(g_err, sizeof(g_err), "no hipBLASLt plan / algorithm %d for layout %d %lldx%lldx%lld", i, layout, M,
                  N, K);
    return -1;
  }
  if (bias && !ok(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)),
                  "BIAS_POINTER"))
    return -2;
  const float alpha = 1.f;
  // library A = weight-side operand, library B = activation-side operand (see layout comment)
  const void* A = op_b;
  const void* B = op_a;
  const hipblasStatus_t st = hipblasLtMatmul(h, p->desc, &alpha, A, p->la, B, p->lb,
                                             &beta, d, p->ld, d, p->ld, &p->algos[i].algo, ws, (size_t)ws_bytes, s);
  return ok(st, "hipblasLtMatmul") ? 0 : (int)st;
}
