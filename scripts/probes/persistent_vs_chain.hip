// Probe (not part of the library): does a PERSISTENT background kernel (one
// launch, grid barriers between its phases) slow a concurrent chain of
// dependent launches less than a background chain of dependent launches does?
// (profiles/README.md round 5: the eigensolver's two reduction chains lose
// ~0.4 ms per ms of overlap in the shared dependent-launch path.)
//
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o persistent_vs_chain.so persistent_vs_chain.hip
//   used by scripts/probes/probe_persistent_vs_chain.py
#include <hip/hip_runtime.h>

namespace {

__global__ __launch_bounds__(64) void tiny_kernel(float* buf) {
  if (threadIdx.x == 0) buf[blockIdx.x] += 1.f;
}

// `phases` grid barriers over a monotonically increasing arrival counter
// (zeroed by the host before the launch).  Every wait is bounded: after
// ~2^22 polls the workgroup flags `err` and every later wait returns at
// once, so all waves always reach the end.
template <int SLEEP>
__global__ __launch_bounds__(64) void persistent_kernel(unsigned* counter, unsigned* err,
                                                        float* buf, int phases) {
  for (int p = 0; p < phases; ++p) {
    if (threadIdx.x == 0) {
      buf[blockIdx.x] += 1.f;
      __atomic_thread_fence(__ATOMIC_RELEASE);
      __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)(p + 1) * gridDim.x;
      unsigned spins = 0;
      while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) break;
        if (++spins > (1u << 22)) {
          __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(SLEEP);
      }
      __atomic_thread_fence(__ATOMIC_ACQUIRE);
    }
    __syncthreads();
  }
}

float* g_buf = nullptr;
unsigned* g_sync = nullptr;    // [0] counter, [1] err
hipGraphExec_t g_exec[2] = {nullptr, nullptr};   // two chains never share an exec
int g_n[2] = {0, 0};

}  // namespace

extern "C" {

int pvc_init() {
  if (g_buf) return 0;
  if (hipMalloc(&g_buf, 4096 * sizeof(float)) != hipSuccess) return 1;
  if (hipMemset(g_buf, 0, 4096 * sizeof(float)) != hipSuccess) return 2;
  if (hipMalloc(&g_sync, 2 * sizeof(unsigned)) != hipSuccess) return 3;
  return (int)hipMemset(g_sync, 0, 2 * sizeof(unsigned));
}

// chain `which` (0 / 1): n dependent one-workgroup launches, captured once, replayed on `s`
int pvc_chain(hipStream_t s, int n, int which) {
  if (which < 0 || which > 1) return 9;
  if (!g_exec[which] || g_n[which] != n) {
    hipStream_t cap;
    if (hipStreamCreateWithFlags(&cap, hipStreamNonBlocking) != hipSuccess) return 10;
    hipGraph_t g;
    if (hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal) != hipSuccess) return 11;
    for (int i = 0; i < n; ++i)
      hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, cap, g_buf + 512 * which);
    if (hipStreamEndCapture(cap, &g) != hipSuccess) return 12;
    if (hipGraphInstantiate(&g_exec[which], g, nullptr, nullptr, 0) != hipSuccess) return 13;
    hipGraphDestroy(g);
    hipStreamDestroy(cap);
    g_n[which] = n;
  }
  return (int)hipGraphLaunch(g_exec[which], s);
}

// one persistent launch of `grid` workgroups (<= 256: one per CU) running `phases` barriers
// sleep: s_sleep argument between polls (1, 8 or 32; ~64 cycles each)
int pvc_persistent(hipStream_t s, int phases, int grid, int sleep) {
  if (grid < 1 || grid > 256) return 20;
  if (hipMemsetAsync(g_sync, 0, 2 * sizeof(unsigned), s) != hipSuccess) return 21;
  if (sleep == 32)
    hipLaunchKernelGGL(persistent_kernel<32>, dim3(grid), dim3(64), 0, s, g_sync, g_sync + 1,
                       g_buf + 1024, phases);
  else if (sleep == 8)
    hipLaunchKernelGGL(persistent_kernel<8>, dim3(grid), dim3(64), 0, s, g_sync, g_sync + 1,
                       g_buf + 1024, phases);
  else
    hipLaunchKernelGGL(persistent_kernel<1>, dim3(grid), dim3(64), 0, s, g_sync, g_sync + 1,
                       g_buf + 1024, phases);
  return (int)hipGetLastError();
}

// err flag of the last persistent launch (call after synchronising)
int pvc_err() {
  unsigned h[2] = {0, 0};
  if (hipMemcpy(h, g_sync, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (int)h[1];
}

}
