// Diagnostic: how long the dispatcher takes to start every workgroup of a
// grid shaped like the step kernels', and what the kernel's fixed cost is
// beyond its own work.  Each workgroup's first lane stamps s_memrealtime
// (100 MHz) at entry, then the workgroup spins for SPIN_US and stamps again;
// the host prints, per shape, the spread of the entry stamps (median / max
// after the first) and the event-timed launch minus the spin.
//   hipcc --offload-arch=gfx950 -O2 -o dispatch_ramp dispatch_ramp.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int SPIN_TICKS = 1000;  // 10 us at 100 MHz

// VG: allocate at least VG VGPRs (a clobber of v[VG-1]); LDS: bytes of static LDS
template <int VG, int LDS>
__global__ void k_ramp(unsigned long long* st, const double* cold, double* sink) {
  __shared__ double lds[LDS / 8 > 0 ? LDS / 8 : 1];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if constexpr (VG > 32) {
    if constexpr (VG == 160) asm volatile("" ::: "v159");
    if constexpr (VG == 128) asm volatile("" ::: "v127");
    if constexpr (VG == 96) asm volatile("" ::: "v95");
    if constexpr (VG == 64) asm volatile("" ::: "v63");
  }
  double x = 0.;
  if (cold) x = cold[(size_t)blockIdx.x * blockDim.x + threadIdx.x];  // a cold load, like the prologue's
  if (LDS > 0) {
    lds[threadIdx.x % (LDS / 8)] = x;
    __syncthreads();
    x += lds[(threadIdx.x + 1) % (LDS / 8)];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t1;
  while (t - t1 < SPIN_TICKS) t = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    st[blockIdx.x * 4 + 0] = t0;
    st[blockIdx.x * 4 + 1] = t1;
    st[blockIdx.x * 4 + 2] = t;
    st[blockIdx.x * 4 + 3] = ((unsigned long long)xcc << 32) | hw;
  }
  if (x == -12345.) sink[0] = x;
}

template <int VG, int LDS>
void run(const char* name, int grid, int block, bool cold_load, unsigned long long* st, double* cold,
         double* sink) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  std::vector<double> dur;
  std::vector<double> med, mx, pro;
  std::vector<unsigned long long> h((size_t)grid * 4);
  for (int r = 0; r < 12; ++r) {
    hipEventRecord(a, 0);
    hipLaunchKernelGGL((k_ramp<VG, LDS>), dim3(grid), dim3(block), 0, 0, st, cold_load ? cold : nullptr, sink);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
    if (r < 2) continue;  // warm
    std::vector<unsigned long long> t0(grid), p(grid);
    for (int i = 0; i < grid; ++i) {
      t0[i] = h[i * 4];
      p[i] = h[i * 4 + 1] - h[i * 4];
    }
    const unsigned long long m0 = *std::min_element(t0.begin(), t0.end());
    std::vector<unsigned long long> rel(grid);
    for (int i = 0; i < grid; ++i) rel[i] = t0[i] - m0;
    std::sort(rel.begin(), rel.end());
    std::sort(p.begin(), p.end());
    med.push_back(rel[grid / 2] * 0.01);
    mx.push_back(rel[grid - 1] * 0.01);
    pro.push_back(p[grid / 2] * 0.01);
    dur.push_back(ms * 1e3);
  }
  auto md = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  printf("{\"shape\": \"%s\", \"grid\": %d, \"block\": %d, \"vgpr\": %d, \"lds\": %d, \"cold_load\": %d, "
         "\"start_spread_median_us\": %.2f, \"start_spread_max_us\": %.2f, \"entry_to_spin_us\": %.2f, "
         "\"launch_us\": %.2f, \"fixed_us\": %.2f}\n",
         name, grid, block, VG, LDS, (int)cold_load, md(med), md(mx), md(pro), md(dur), md(dur) - SPIN_TICKS * 0.01);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

int main() {
  unsigned long long* st;
  double *cold, *sink;
  hipMalloc(&st, 4096 * 4 * 8);
  hipMalloc(&cold, (size_t)4096 * 1024 * 8 * 2);
  hipMalloc(&sink, 64);
  hipMemset(cold, 0, (size_t)4096 * 1024 * 8 * 2);
  run<160, 64000>("trio-like 256x768", 256, 768, true, st, cold, sink);
  run<160, 64000>("trio-like 256x768 no load", 256, 768, false, st, cold, sink);
  run<32, 0>("256x768 light", 256, 768, false, st, cold, sink);
  run<128, 32000>("256x1024 (4 waves/SIMD)", 256, 1024, true, st, cold, sink);
  run<160, 32000>("512x384", 512, 384, true, st, cold, sink);
  run<160, 16000>("1024x192", 1024, 192, true, st, cold, sink);
  run<96, 0>("1024x256 single-role-like", 1024, 256, true, st, cold, sink);
  run<64, 0>("2048x256", 2048, 256, true, st, cold, sink);
  run<32, 0>("256x256 light", 256, 256, false, st, cold, sink);
  hipFree(st);
  hipFree(cold);
  hipFree(sink);
  return 0;
}
