// Every hipBLASLt solution for the config #5 encoder-side GEMM shapes, timed one by one against
// the library's top heuristic pick (the one torch.mm gets).  Row-major notation as the engine
// issues them: C[M,N] (+)= op(A) . op(B), bf16 operands, fp32 accumulate, fp32 or bf16 output.
//
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/micro/hipblaslt_probe.cpp -lhipblaslt -o build/hipblaslt_probe
//   build/hipblaslt_probe [rows]        (rows = batch x T, default 819200)
//
// Prints one JSON line per shape: heuristic-pick us, best us, the best solution's index/name.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    auto _e = (x);                                                                             \
    if ((int)_e != 0) {                                                                        \
      std::fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, (int)_e);               \
      std::exit(1);                                                                            \
    }                                                                                          \
  } while (0)

struct Shape {
  const char* name;
  bool ta, tb;  // row-major: A stored [K,M] if ta, B stored [N,K] if tb
  long M, N, K;
  bool bf16_out;
  float beta;
};

static hipblasLtHandle_t H;

// random bf16 in about [-0.1, 0.1] (a hash of the index): constant operands clock higher
__global__ void fill_rand(unsigned short* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 15; x *= 2246822519u; x ^= x >> 13; x *= 3266489917u; x ^= x >> 16;
    float f = ((x & 0xffffff) / 16777216.f - 0.5f) * 0.2f;
    unsigned u = __float_as_uint(f);
    p[i] = (unsigned short)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
  }
}
static void* WS;
static const size_t WS_BYTES = 256ull << 20;

struct Prob {
  hipblasLtMatmulDesc_t desc;
  hipblasLtMatrixLayout_t la, lb, lc;
  hipblasOperation_t opa, opb;
};

// column-major call: D'[N,M] = op(B') . op(A') with B' = row-major B, A' = row-major A
static Prob make(const Shape& s) {
  Prob p;
  hipDataType od = s.bf16_out ? HIP_R_16BF : HIP_R_32F;
  CK(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  p.opa = s.tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;  // hipblas A = engine B
  p.opb = s.ta ? HIPBLAS_OP_T : HIPBLAS_OP_N;  // hipblas B = engine A
  CK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &p.opa, sizeof(p.opa)));
  CK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &p.opb, sizeof(p.opb)));
  // engine B: [K,N] row-major = col-major [N,K] ld N; transposed: [N,K] row-major = col-major [K,N] ld K
  if (!s.tb) CK(hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, s.N, s.K, s.N));
  else CK(hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, s.K, s.N, s.K));
  if (!s.ta) CK(hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, s.K, s.M, s.K));
  else CK(hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, s.M, s.K, s.M));
  CK(hipblasLtMatrixLayoutCreate(&p.lc, od, s.N, s.M, s.N));
  return p;
}

static float time_algo(const Shape& s, Prob& p, hipblasLtMatmulAlgo_t& algo, void* A, void* B, void* C, int reps) {
  float alpha = 1.f, beta = s.beta;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&]() {
    return hipblasLtMatmul(H, p.desc, &alpha, B, p.la, A, p.lb, &beta, C, p.lc, C, p.lc, &algo, WS, WS_BYTES, 0);
  };
  if (run() != HIPBLAS_STATUS_SUCCESS) return -1.f;
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) run();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms * 1000.f / reps;
}

int main(int argc, char** argv) {
  long R = argc > 1 ? std::atol(argv[1]) : 819200;
  double budget_s = argc > 2 ? std::atof(argv[2]) : 45.0;
  const long Hd = 512;
  std::vector<Shape> shapes = {
      {"fwd_gx_l2", false, false, R, 4 * Hd, 2 * Hd, false, 0.f},
      {"fwd_F_bf16", false, false, R, 2 * Hd, 2 * Hd, true, 0.f},
      {"dx_l2", false, true, R, 2 * Hd, 4 * Hd, false, 0.f},
      {"dE_addmm", false, true, R, 2 * Hd, 2 * Hd, false, 1.f},
      {"wg_x2", true, false, 2 * Hd, 4 * Hd, R, false, 0.f},
      {"wg_h", true, false, Hd, 4 * Hd, R, false, 0.f},
      {"wg_wh", true, false, 2 * Hd, 2 * Hd, R, false, 0.f},
      {"dx_l1", false, true, R, 128, 4 * Hd, false, 0.f},
      {"wg_x1", true, false, 128, 4 * Hd, R, false, 0.f},
  };
  CK(hipblasLtCreate(&H));
  CK(hipMalloc(&WS, WS_BYTES));
  size_t maxA = R * 4 * Hd * 2, maxC = R * 4 * Hd * 4;
  void *A, *B, *C;
  CK(hipMalloc(&A, maxA));
  CK(hipMalloc(&B, maxA));
  CK(hipMalloc(&C, maxC));
  hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, (unsigned short*)A, maxA / 2, 17u);
  hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, (unsigned short*)B, maxA / 2, 91u);
  CK(hipDeviceSynchronize());
  CK(hipMemset(C, 0, maxC));
  for (auto& s : shapes) {
    Prob p = make(s);
    double flop = 2.0 * s.M * s.N * s.K;
    hipblasLtMatmulPreference_t pref;
    CK(hipblasLtMatmulPreferenceCreate(&pref));
    uint64_t wsb = WS_BYTES;
    CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
    hipblasLtMatmulHeuristicResult_t hr[1];
    int got = 0;
    CK(hipblasLtMatmulAlgoGetHeuristic(H, p.desc, p.la, p.lb, p.lc, p.lc, pref, 1, hr, &got));
    float th = got ? time_algo(s, p, hr[0].algo, A, B, C, 5) : -1.f;
    int hidx = got ? hipblaslt_ext::getIndexFromAlgo(hr[0].algo) : -1;
    std::vector<hipblasLtMatmulHeuristicResult_t> all;
    hipblaslt_ext::getAllAlgos(H, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, p.opa, p.opb, HIP_R_16BF, HIP_R_16BF,
                               s.bf16_out ? HIP_R_16BF : HIP_R_32F, s.bf16_out ? HIP_R_16BF : HIP_R_32F,
                               HIPBLAS_COMPUTE_32F, all);
    float alpha = 1.f, beta = s.beta;
    std::vector<std::pair<float, int>> res;
    int tried = 0, supported = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (size_t i = 0; i < all.size(); ++i) {
      size_t need = 0;
      if (hipblaslt_ext::matmulIsAlgoSupported(H, p.desc, &alpha, p.la, p.lb, &beta, p.lc, p.lc, all[i].algo, need) !=
              HIPBLAS_STATUS_SUCCESS ||
          need > WS_BYTES)
        continue;
      ++supported;
      // a quick single run screens out the slow half before the timed reps
      float t1 = time_algo(s, p, all[i].algo, A, B, C, 1);
      ++tried;
      if (t1 > 0 && (th < 0 || t1 < 1.3f * th)) {
        float t = time_algo(s, p, all[i].algo, A, B, C, 3);
        if (t > 0) res.push_back({t, (int)i});
      }
      double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (tried % 50 == 0) std::fprintf(stderr, "  %s: %d tried, %.1fs\n", s.name, tried, el);
      if (el > budget_s) break;
    }
    std::sort(res.begin(), res.end());
    float tb = res.empty() ? -1.f : res[0].first;
    std::string name = res.empty() ? "" : hipblaslt_ext::getSolutionNameFromAlgo(H, all[res[0].second].algo);
    int bidx = res.empty() ? -1 : hipblaslt_ext::getIndexFromAlgo(all[res[0].second].algo);
    // re-time the two with more reps, side by side
    if (!res.empty()) {
      th = got ? time_algo(s, p, hr[0].algo, A, B, C, 10) : -1.f;
      tb = time_algo(s, p, all[res[0].second].algo, A, B, C, 10);
    }
    std::printf(
        "{\"shape\": \"%s\", \"M\": %ld, \"N\": %ld, \"K\": %ld, \"heur_us\": %.1f, \"heur_TF\": %.0f, \"heur_idx\": %d, "
        "\"best_us\": %.1f, \"best_TF\": %.0f, \"best_idx\": %d, \"algos\": %zu, \"supported\": %d, \"tried\": %d, "
        "\"best_name\": \"%s\", \"top5\": [",
        s.name, s.M, s.N, s.K, th, flop / (th * 1e-6) / 1e12, hidx, tb, flop / (tb * 1e-6) / 1e12, bidx, all.size(),
        supported, tried, name.c_str());
    for (size_t j = 0; j < res.size() && j < 5; ++j)
      std::printf("%s[%d, %.1f]", j ? ", " : "", hipblaslt_ext::getIndexFromAlgo(all[res[j].second].algo),
                  res[j].first);
    std::printf("]}\n");
    std::fflush(stdout);
    hipblasLtMatmulPreferenceDestroy(pref);
  }
  return 0;
}
