// Probe: rocSOLVER syevd / sytrd / stedc / ormtr cost split and the effect of
// the fill mode (upper vs lower) at the large K-FAC factor sizes on gfx950.
// hipcc -O2 --offload-arch=gfx950 probe_fill.cpp -lrocsolver -lrocblas -o probe_fill
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { auto e = (x); if (e != hipSuccess) { printf("hip err %d line %d\n", (int)e, __LINE__); exit(1);} } while (0)

static void make_spd(std::vector<float>& A, int n, int rank, unsigned seed) {
  std::mt19937 g(seed); std::normal_distribution<float> nd;
  std::vector<float> X((size_t)rank * n);
  for (auto& v : X) v = nd(g);
  for (int i = 0; i < n; ++i) for (int j = 0; j <= i; ++j) {
    double s = 0; for (int k = 0; k < rank; ++k) s += (double)X[(size_t)k * n + i] * X[(size_t)k * n + j];
    float v = (float)(s / rank) + (i == j ? 0.05f : 0.f);
    A[(size_t)i * n + j] = v; A[(size_t)j * n + i] = v;
  }
}

int main() {
  rocblas_handle h; rocblas_create_handle(&h);
  hipStream_t st; CK(hipStreamCreate(&st)); rocblas_set_stream(h, st);
  int sizes[] = {1024, 2304, 4608};
  for (int n : sizes) {
    int batch = (n == 4608) ? 3 : 6;
    std::vector<float> A((size_t)n * n);
    make_spd(A, n, 64, n);
    size_t nn = (size_t)n * n;
    float *dA, *dA0, *dD, *dE, *dW, *dC; int* dinfo;
    CK(hipMalloc(&dA, nn * 4 * batch)); CK(hipMalloc(&dA0, nn * 4 * batch)); CK(hipMalloc(&dC, nn * 4));
    CK(hipMalloc(&dD, n * 4 * batch)); CK(hipMalloc(&dE, n * 4 * batch)); CK(hipMalloc(&dW, n * 4 * batch));
    CK(hipMalloc(&dinfo, 4 * batch));
    for (int b = 0; b < batch; ++b) CK(hipMemcpy(dA0 + nn * b, A.data(), nn * 4, hipMemcpyHostToDevice));
    auto run = [&](const char* name, int bc, auto fn) {
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemcpyAsync(dA, dA0, nn * 4 * bc, hipMemcpyDeviceToDevice, st));
        CK(hipStreamSynchronize(st));
        auto t0 = std::chrono::high_resolution_clock::now();
        fn(bc);
        CK(hipStreamSynchronize(st));
        double ms = std::chrono::duration<double, std::milli>(std::chrono::high_resolution_clock::now() - t0).count();
        if (rep == 1) printf("n=%5d batch=%d %-14s %9.2f ms\n", n, bc, name, ms);
      }
      fflush(stdout);
    };
    for (int bc : {1, batch}) {
      run("syevd upper", bc, [&](int b) { rocsolver_ssyevd_strided_batched(h, rocblas_evect_original, rocblas_fill_upper, n, dA, n, nn, dD, n, dE, n, dinfo, b); });
      run("syevd lower", bc, [&](int b) { rocsolver_ssyevd_strided_batched(h, rocblas_evect_original, rocblas_fill_lower, n, dA, n, nn, dD, n, dE, n, dinfo, b); });
      run("sytrd upper", bc, [&](int b) { rocsolver_ssytrd_strided_batched(h, rocblas_fill_upper, n, dA, n, nn, dD, n, dE, n, dW, n, b); });
      run("sytrd lower", bc, [&](int b) { rocsolver_ssytrd_strided_batched(h, rocblas_fill_lower, n, dA, n, nn, dD, n, dE, n, dW, n, b); });
    }
    // ormtr cost on top of a lower sytrd
    CK(hipMemcpy(dA, dA0, nn * 4, hipMemcpyDeviceToDevice));
    rocsolver_ssytrd(h, rocblas_fill_lower, n, dA, n, dD, dE, dW);
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemcpy(dC, dA0, nn * 4, hipMemcpyDeviceToDevice));
      CK(hipStreamSynchronize(st));
      auto t0 = std::chrono::high_resolution_clock::now();
      rocsolver_sormtr(h, rocblas_side_left, rocblas_fill_lower, rocblas_operation_none, n, n, dA, n, dW, dC, n);
      CK(hipStreamSynchronize(st));
      double ms = std::chrono::duration<double, std::milli>(std::chrono::high_resolution_clock::now() - t0).count();
      if (rep == 1) printf("n=%5d ormtr lower    %9.2f ms\n", n, ms);
    }
    hipFree(dA); hipFree(dA0); hipFree(dD); hipFree(dE); hipFree(dW); hipFree(dC); hipFree(dinfo);
  }
  return 0;
}
