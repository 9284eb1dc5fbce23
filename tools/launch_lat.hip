// Diagnostic: the platform's launch and synchronisation costs on this box,
// outside Python: host time per hipLaunchKernelGGL (empty kernel, 256
// workgroups; small and ~600-byte argument blocks), launch + synchronise
// round trips (stream / device / event), and the same kernel replayed from an
// instantiated hipGraph.   hipcc --offload-arch=gfx950 -O2 -o launch_lat launch_lat.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>
#include <algorithm>

struct Big {
  double v[76];
};

__global__ void k_small(int* p, int n) {
  if (p && blockIdx.x * blockDim.x + threadIdx.x < (unsigned)n) p[0] = 1;
}
__global__ void k_big(Big b, int* p) {
  if (p && b.v[threadIdx.x & 63] == -1.0) p[0] = 1;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <typename F>
static double median_us(F f, int reps) {
  std::vector<double> t;
  for (int i = 0; i < reps; ++i) {
    const double a = now_us();
    f();
    t.push_back(now_us() - a);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  int* d = nullptr;
  (void)hipMalloc(&d, 64);
  Big b{};
  for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, s, d, 0);
  (void)hipStreamSynchronize(s);
  // host cost per launch (queue not drained: 200 launches back to back)
  double t0 = now_us();
  for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, s, d, 0);
  const double small_call = (now_us() - t0) / 200;
  (void)hipStreamSynchronize(s);
  t0 = now_us();
  for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s, b, d);
  const double big_call = (now_us() - t0) / 200;
  (void)hipStreamSynchronize(s);
  // round trips
  const double rt_stream = median_us([&] {
    hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s, b, d);
    (void)hipStreamSynchronize(s);
  }, 200);
  const double rt_device = median_us([&] {
    hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s, b, d);
    (void)hipDeviceSynchronize();
  }, 200);
  hipEvent_t ev;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  const double rt_event = median_us([&] {
    hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s, b, d);
    (void)hipEventRecord(ev, s);
    (void)hipEventSynchronize(ev);
  }, 200);
  const double rt_null = median_us([&] {
    hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, 0, b, d);
    (void)hipDeviceSynchronize();
  }, 200);
  // graph of one kernel
  hipGraph_t g;
  hipGraphExec_t ge;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, s, b, d);
  (void)hipStreamEndCapture(s, &g);
  (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int i = 0; i < 20; ++i) (void)hipGraphLaunch(ge, s);
  (void)hipStreamSynchronize(s);
  t0 = now_us();
  for (int i = 0; i < 200; ++i) (void)hipGraphLaunch(ge, s);
  const double graph_call = (now_us() - t0) / 200;
  (void)hipStreamSynchronize(s);
  const double rt_graph = median_us([&] {
    (void)hipGraphLaunch(ge, s);
    (void)hipStreamSynchronize(s);
  }, 200);
  const double idle_sync = median_us([&] { (void)hipStreamSynchronize(s); }, 200);
  std::printf("{\"launch_call_small_us\": %.2f, \"launch_call_big_us\": %.2f, \"graph_launch_call_us\": %.2f, "
              "\"roundtrip_stream_sync_us\": %.2f, \"roundtrip_device_sync_us\": %.2f, "
              "\"roundtrip_event_sync_us\": %.2f, \"roundtrip_null_stream_us\": %.2f, "
              "\"roundtrip_graph_us\": %.2f, \"idle_stream_sync_us\": %.2f}\n",
              small_call, big_call, graph_call, rt_stream, rt_device, rt_event, rt_null, rt_graph, idle_sync);
  return 0;
}
