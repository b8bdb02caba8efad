// Captured-graph memset nodes -> fill kernels.
//
// On the ROCm 7.2 runtime of this image a memset node of a captured hipGraph
// does not reliably clear its destination on replay (found first in the
// eigensolver's back-transformation graph, scripts/probes/probe_graph_memset.py).
// Libraries that zero a buffer with hipMemsetAsync before accumulating into it
// then compute garbage when the stream is captured: MIOpen's channels_last
// weight-gradient algorithm for ResNet-50's layer2.0.conv1 (picked with
// cudnn.benchmark) adds its partial sums onto whatever the previous user of
// the memory left (scripts/probes/debug_fb_graph.py POKE mode: a buffer filled
// with 1e30 and freed between replays shows up as a 1e30 gradient; profiles/
// README.md).  graphs.GraphedTrainStep and KFAC's tail graph therefore capture
// with keep_graph=True and run every graph through kfac_graph_fix_memsets
// before instantiating it: each memset node is replaced by a kernel node that
// writes the same pattern, with the same dependencies.
#include "common.h"

#include <vector>

namespace {

// pattern word: byte at offset o from the memset's dst is byte (o % 4) of `word`
// (element sizes 1, 2, 4 all have a period dividing 4)
__device__ __forceinline__ unsigned rot_word(unsigned word, size_t off) {
  const unsigned s = (unsigned)(off & 3) * 8u;
  return s ? ((word >> s) | (word << (32u - s))) : word;
}

__global__ __launch_bounds__(256) void fill_rows_kernel(unsigned char* __restrict__ dst, size_t pitch,
                                                        size_t row_bytes, size_t rows,
                                                        unsigned word) {
  for (size_t r = 0; r < rows; ++r) {
    unsigned char* base = dst + r * pitch;
    const size_t addr = (size_t)base;
    // [head, head + nvec*16) is 16-byte aligned
    size_t head = (16 - (addr & 15)) & 15;
    if (head > row_bytes) head = row_bytes;
    const size_t nvec = (row_bytes - head) / 16;
    const size_t tail0 = head + nvec * 16;
    const size_t tid = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t nthr = (size_t)gridDim.x * 256;
    if (tid < head) base[tid] = (unsigned char)(word >> ((tid & 3) * 8));
    const unsigned w = rot_word(word, head);
    const uint4 v = make_uint4(w, w, w, w);
    uint4* vp = (uint4*)(base + head);
    for (size_t i = tid; i < nvec; i += nthr) vp[i] = v;
    for (size_t o = tail0 + tid; o < row_bytes; o += nthr)
      base[o] = (unsigned char)(word >> ((o & 3) * 8));
  }
}

int fix_graph(hipGraph_t g, int replace, int depth, long long* stats) {
  if (depth > 8) return -30;
  size_t n = 0;
  if (hipGraphGetNodes(g, nullptr, &n) != hipSuccess) return -31;
  std::vector<hipGraphNode_t> nodes(n);
  if (n && hipGraphGetNodes(g, nodes.data(), &n) != hipSuccess) return -31;
  for (hipGraphNode_t node : nodes) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(node, &t) != hipSuccess) return -32;
    if (t == hipGraphNodeTypeGraph) {
      hipGraph_t child = nullptr;
      if (hipGraphChildGraphNodeGetGraph(node, &child) != hipSuccess) return -33;
      int e = fix_graph(child, replace, depth + 1, stats);
      if (e) return e;
      continue;
    }
    if (t != hipGraphNodeTypeMemset) continue;
    hipMemsetParams p;
    if (hipGraphMemsetNodeGetParams(node, &p) != hipSuccess) return -34;
    const size_t es = p.elementSize;
    if (es != 1 && es != 2 && es != 4) return -35;
    const size_t row_bytes = p.width * es;
    const size_t rows = p.height ? p.height : 1;
    stats[0] += 1;
    stats[1] += (long long)(row_bytes * rows);
    if (!replace) continue;
    unsigned v = p.value;
    unsigned word = es == 4 ? v : es == 2 ? ((v & 0xffffu) | ((v & 0xffffu) << 16))
                                           : (v & 0xffu) * 0x01010101u;
    size_t nd = 0, nx = 0;
    if (hipGraphNodeGetDependencies(node, nullptr, &nd) != hipSuccess) return -36;
    if (hipGraphNodeGetDependentNodes(node, nullptr, &nx) != hipSuccess) return -36;
    std::vector<hipGraphNode_t> deps(nd), outs(nx);
    if (nd && hipGraphNodeGetDependencies(node, deps.data(), &nd) != hipSuccess) return -36;
    if (nx && hipGraphNodeGetDependentNodes(node, outs.data(), &nx) != hipSuccess) return -36;
    unsigned char* dst = (unsigned char*)p.dst;
    size_t pitch = p.pitch ? p.pitch : row_bytes;
    size_t chunks = (row_bytes + 4095) / 4096;   // 256 lanes x 16 B per block
    unsigned blocks = (unsigned)(chunks < 1 ? 1 : chunks > 2048 ? 2048 : chunks);
    void* args[] = {&dst, &pitch, (void*)&row_bytes, (void*)&rows, &word};
    hipKernelNodeParams kp = {};
    kp.func = (void*)fill_rows_kernel;
    kp.gridDim = dim3(blocks);
    kp.blockDim = dim3(256);
    kp.sharedMemBytes = 0;
    kp.kernelParams = args;
    kp.extra = nullptr;
    hipGraphNode_t kn;
    if (hipGraphAddKernelNode(&kn, g, nd ? deps.data() : nullptr, nd, &kp) != hipSuccess)
      return -37;
    for (size_t i = 0; i < nx; ++i)
      if (hipGraphAddDependencies(g, &kn, &outs[i], 1) != hipSuccess) return -38;
    if (hipGraphDestroyNode(node) != hipSuccess) return -39;
    stats[2] += 1;
  }
  return 0;
}

}  // namespace

// stats[0] memset nodes found, stats[1] bytes they set, stats[2] nodes replaced.
// `graph` is a captured, not yet instantiated hipGraph_t.
KFAC_API int kfac_graph_fix_memsets(void* graph, int replace, long long* stats) {
  stats[0] = stats[1] = stats[2] = 0;
  int e = fix_graph((hipGraph_t)graph, replace, 0, stats);
  (void)hipGetLastError();
  return e;
}

// Cross-graph signalling: an event recorded with hipEventRecordExternal while
// a stream is being captured becomes an external event-record node of that
// graph, and hipStreamWaitEvent(..., hipEventWaitExternal) an external wait
// node of another graph, so two graphs replayed on two streams can hand off
// in the MIDDLE of the first one (torch refuses external events on ROCm).
KFAC_API void* kfac_event_create() {
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
  return (void*)e;
}
KFAC_API int kfac_event_destroy(void* e) { return (int)hipEventDestroy((hipEvent_t)e); }
// During a capture the node is added by hand after the stream's current
// capture dependencies (hipEventRecordWithFlags(.., hipEventRecordExternal)
// returns hipErrorInvalidValue under capture on this ROCm); outside a
// capture these are the plain record / wait.
namespace {
int add_capture_node(hipStream_t s, void* e, bool record, bool* captured) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t ndeps = 0;
  hipError_t r = hipStreamGetCaptureInfo_v2(s, &st, &id, &g, &deps, &ndeps);
  if (r != hipSuccess) return (int)r;
  *captured = st == hipStreamCaptureStatusActive;
  if (!*captured) return 0;
  hipGraphNode_t node = nullptr;
  r = record ? hipGraphAddEventRecordNode(&node, g, deps, ndeps, (hipEvent_t)e)
             : hipGraphAddEventWaitNode(&node, g, deps, ndeps, (hipEvent_t)e);
  if (r != hipSuccess) return (int)r;
  return (int)hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies);
}
}  // namespace

KFAC_API int kfac_event_record_external(void* e, hipStream_t s) {
  bool cap = false;
  const int r = add_capture_node(s, e, true, &cap);
  if (r || cap) return r;
  return (int)hipEventRecord((hipEvent_t)e, s);
}
KFAC_API int kfac_stream_wait_external(hipStream_t s, void* e) {
  bool cap = false;
  const int r = add_capture_node(s, e, false, &cap);
  if (r || cap) return r;
  return (int)hipStreamWaitEvent(s, (hipEvent_t)e, 0);
}
