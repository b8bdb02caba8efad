// Probe: rocSOLVER symmetric eigensolver variants at K-FAC factor sizes on gfx950.
// hipcc -O2 --offload-arch=gfx950 probe_rocsolver.cpp -lrocsolver -lrocblas -o probe_rocsolver
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>

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

int main(int argc, char** argv) {
  rocblas_handle h; rocblas_create_handle(&h);
  hipStream_t st; CK(hipStreamCreate(&st)); rocblas_set_stream(h, st);
  int sizes[] = {256, 512, 1024, 2048, 2304, 4608};
  for (int n : sizes) {
    int batch = (n == 4608) ? 3 : 6;
    std::vector<float> A((size_t)n * n);
    make_spd(A, n, n < 1024 ? n / 2 : 512, n);
    size_t nn = (size_t)n * n;
    float *dA, *dA0, *dD, *dE, *dres, *dW; int *dinfo, *dsw;
    CK(hipMalloc(&dA, nn * 4 * batch)); CK(hipMalloc(&dA0, nn * 4 * batch));
    CK(hipMalloc(&dD, n * 4 * batch)); CK(hipMalloc(&dE, n * 4 * batch)); CK(hipMalloc(&dW, n * 4 * batch));
    CK(hipMalloc(&dres, 4 * batch)); CK(hipMalloc(&dinfo, 4 * batch)); CK(hipMalloc(&dsw, 4 * batch));
    for (int b = 0; b < batch; ++b) CK(hipMemcpy(dA0 + nn * b, A.data(), nn * 4, hipMemcpyHostToDevice));
    auto run = [&](const char* name, int bc, auto fn) {
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemcpyAsync(dA, dA0, nn * 4 * bc, hipMemcpyDeviceToDevice, st));
        CK(hipStreamSynchronize(st));
        auto t0 = std::chrono::high_resolution_clock::now();
        fn(bc);
        CK(hipStreamSynchronize(st));
        double ms = std::chrono::duration<double, std::milli>(std::chrono::high_resolution_clock::now() - t0).count();
        if (rep == 1) printf("n=%5d batch=%d %-22s %9.2f ms\n", n, bc, name, ms);
      }
      fflush(stdout);
    };
    for (int bc : {1, batch}) {
      run("syevd", bc, [&](int b) { rocsolver_ssyevd_strided_batched(h, rocblas_evect_original, rocblas_fill_upper, n, dA, n, nn, dD, n, dE, n, dinfo, b); });
      run("syevdj", bc, [&](int b) { rocsolver_ssyevdj_strided_batched(h, rocblas_evect_original, rocblas_fill_upper, n, dA, n, nn, dD, n, dinfo, b); });
      if (n <= 1024)
        run("syevj(tol1e-6,20)", bc, [&](int b) { rocsolver_ssyevj_strided_batched(h, rocblas_esort_ascending, rocblas_evect_original, rocblas_fill_upper, n, dA, n, nn, 1e-6f, dres, 20, dsw, dW, n, dinfo, b); });
      run("sytrd", bc, [&](int b) { rocsolver_ssytrd_strided_batched(h, rocblas_fill_upper, n, dA, n, nn, dD, n, dE, n, dW, n, b); });
    }
    // stedc alone on a tridiagonal from sytrd
    CK(hipMemcpy(dA, dA0, nn * 4, hipMemcpyDeviceToDevice));
    rocsolver_ssytrd(h, rocblas_fill_upper, n, dA, n, dD, dE, dW);
    CK(hipStreamSynchronize(st));
    std::vector<float> D(n), E(n);
    CK(hipMemcpy(D.data(), dD, n * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(E.data(), dE, n * 4, hipMemcpyDeviceToHost));
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemcpy(dD, D.data(), n * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(dE, E.data(), n * 4, hipMemcpyHostToDevice));
      auto t0 = std::chrono::high_resolution_clock::now();
      rocsolver_sstedc(h, rocblas_evect_tridiagonal, n, dD, dE, dA, n, dinfo);
      CK(hipStreamSynchronize(st));
      double ms = std::chrono::duration<double, std::milli>(std::chrono::high_resolution_clock::now() - t0).count();
      if (rep == 1) printf("n=%5d stedc(tridiag evect) %9.2f ms\n", n, ms);
    }
    hipFree(dA); hipFree(dA0); hipFree(dD); hipFree(dE); hipFree(dres); hipFree(dinfo); hipFree(dsw); hipFree(dW);
  }
  return 0;
}
