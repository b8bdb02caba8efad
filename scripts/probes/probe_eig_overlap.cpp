// Probe: do concurrent rocSOLVER syevd calls on different streams overlap on gfx950?
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>
#include <random>

struct Job { int n, batch; float *A, *A0, *D, *E; int* info; hipStream_t s; rocblas_handle h; };

static void setup(Job& j, int n, int batch) {
  j.n = n; j.batch = batch;
  size_t nn = (size_t)n * n;
  hipMalloc(&j.A, nn * 4 * batch); hipMalloc(&j.A0, nn * 4 * batch);
  hipMalloc(&j.D, n * 4 * batch); hipMalloc(&j.E, n * 4 * batch); hipMalloc(&j.info, 4 * batch);
  std::vector<float> h(nn);
  std::mt19937 g(n); std::normal_distribution<float> nd;
  // diagonally dominant-ish SPD test matrix: cheap to build
  for (int i = 0; i < n; ++i) for (int k = 0; k <= i; ++k) { float v = nd(g) / n; if (i == k) v += 1.f + i * 1e-3f; h[(size_t)i*n+k] = v; h[(size_t)k*n+i] = v; }
  for (int b = 0; b < batch; ++b) hipMemcpy(j.A0 + nn * b, h.data(), nn * 4, hipMemcpyHostToDevice);
  hipStreamCreate(&j.s); rocblas_create_handle(&j.h); rocblas_set_stream(j.h, j.s);
}
static void run(Job& j) {
  size_t nn = (size_t)j.n * j.n;
  hipMemcpyAsync(j.A, j.A0, nn * 4 * j.batch, hipMemcpyDeviceToDevice, j.s);
  rocsolver_ssyevd_strided_batched(j.h, rocblas_evect_original, rocblas_fill_upper, j.n, j.A, j.n, nn, j.D, j.n, j.E, j.n, j.info, j.batch);
  hipStreamSynchronize(j.s);
}
static double ms_since(std::chrono::high_resolution_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::high_resolution_clock::now() - t0).count();
}
int main() {
  std::vector<Job> jobs(4);
  setup(jobs[0], 4608, 3); setup(jobs[1], 2304, 6); setup(jobs[2], 2048, 6); setup(jobs[3], 1024, 6);
  for (auto& j : jobs) run(j);  // warm
  double solo[4];
  for (int i = 0; i < 4; ++i) { auto t0 = std::chrono::high_resolution_clock::now(); run(jobs[i]); solo[i] = ms_since(t0); printf("solo n=%d x%d: %.1f ms\n", jobs[i].n, jobs[i].batch, solo[i]); }
  for (int k = 2; k <= 4; ++k) {
    auto t0 = std::chrono::high_resolution_clock::now();
    std::vector<std::thread> th;
    for (int i = 0; i < k; ++i) th.emplace_back([&, i] { run(jobs[i]); });
    for (auto& t : th) t.join();
    double sum = 0, mx = 0; for (int i = 0; i < k; ++i) { sum += solo[i]; mx = solo[i] > mx ? solo[i] : mx; }
    printf("concurrent first %d jobs: %.1f ms (sum of solos %.1f, max %.1f)\n", k, ms_since(t0), sum, mx);
  }
  // same, but single thread issuing to 4 streams (rocSOLVER may block the host)
  {
    auto t0 = std::chrono::high_resolution_clock::now();
    for (auto& j : jobs) {
      size_t nn = (size_t)j.n * j.n;
      hipMemcpyAsync(j.A, j.A0, nn * 4 * j.batch, hipMemcpyDeviceToDevice, j.s);
      rocsolver_ssyevd_strided_batched(j.h, rocblas_evect_original, rocblas_fill_upper, j.n, j.A, j.n, nn, j.D, j.n, j.E, j.n, j.info, j.batch);
    }
    double issue = ms_since(t0);
    for (auto& j : jobs) hipStreamSynchronize(j.s);
    printf("one thread, 4 streams: issue %.1f ms, total %.1f ms\n", issue, ms_since(t0));
  }
  return 0;
}
