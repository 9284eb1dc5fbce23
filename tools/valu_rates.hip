// Diagnostic: issue cost (cycles per wave-instruction, one wave per SIMD and
// three waves per SIMD) of the instruction classes the step kernel is made
// of: v_mad_u64_u32 (Philox), v_xor_b32, v_fma_f64, v_mul_f64, v_rcp_f64,
// v_sqrt_f64, v_add_u32.  Eight independent chains per lane, 256 iterations.
//   hipcc --offload-arch=gfx950 -O3 -o valu_rates valu_rates.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define N_IT 256

template <int OP>
__global__ void k_rate(unsigned long long* out, double* sink, uint32_t seed) {
  uint32_t a[8];
  double f[8];
  for (int i = 0; i < 8; ++i) {
    a[i] = seed + threadIdx.x * 8 + i;
    f[i] = 1.0 + 1e-9 * (threadIdx.x * 8 + i);
  }
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 4
  for (int it = 0; it < N_IT; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (OP == 0) {
        const uint64_t p = (uint64_t)0xD2511F53u * a[i] + i;
        a[i] = (uint32_t)(p >> 32) ^ (uint32_t)p;  // one mad_u64_u32 + one xor
      } else if (OP == 1) {
        a[i] = (a[i] ^ 0x9E3779B9u) + 7u;  // xor + add
      } else if (OP == 2) {
        f[i] = __fma_rn(f[i], 0.999999, 1e-7);
      } else if (OP == 3) {
        f[i] = __builtin_amdgcn_rcp(f[i]) + 1.0;  // v_rcp_f64 + v_add_f64
      } else if (OP == 4) {
        f[i] = __builtin_amdgcn_sqrt(f[i]) + 1.0;  // v_sqrt_f64 + v_add_f64
      } else if (OP == 5) {
        f[i] = f[i] * 1.0000001;
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double acc = 0;
  for (int i = 0; i < 8; ++i) acc += f[i] + a[i];
  sink[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
static void run(const char* name, int waves_per_simd, unsigned long long* d_out, double* sink) {
  const int threads = 256 * waves_per_simd;  // one workgroup on one CU: 4 SIMDs
  hipLaunchKernelGGL(k_rate<OP>, dim3(1), dim3(threads), 0, 0, d_out, sink, 1u);
  (void)hipDeviceSynchronize();
  unsigned long long h[16];
  (void)hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost);
  double mx = 0;
  for (int w = 0; w < threads / 64; ++w) mx = h[w] > mx ? h[w] : mx;
  // cycles per wave-instruction of the measured pair, per SIMD
  std::printf("  \"%s_w%d\": %.2f,\n", name, waves_per_simd, mx / (N_IT * 8.0) / waves_per_simd);
}

int main() {
  unsigned long long* d_out;
  double* sink;
  (void)hipMalloc(&d_out, 16 * sizeof(unsigned long long));
  (void)hipMalloc(&sink, 4096 * sizeof(double));
  std::printf("{\n  \"note\": \"cycles per SIMD per lane-op group (s_memtime ticks), 8 independent chains\",\n");
  for (int w : {1, 3}) {
    run<0>("mad_u64_u32+xor", w, d_out, sink);
    run<1>("xor+add_u32", w, d_out, sink);
    run<2>("fma_f64", w, d_out, sink);
    run<3>("rcp_f64+add_f64", w, d_out, sink);
    run<4>("sqrt_f64+add_f64", w, d_out, sink);
    run<5>("mul_f64", w, d_out, sink);
  }
  std::printf("  \"end\": 0\n}\n");
  return 0;
}
