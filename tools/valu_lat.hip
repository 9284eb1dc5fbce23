// Diagnostic: dependent-chain latency (s_memtime cycles per operation, one
// chain per lane, one wave per SIMD) of the operations on the step kernel's
// critical chains: f64 add / fma / mul, an f64 DPP move + add (one stage of
// the canonical segment sum), an IEEE f64 division, v_rcp_f64, v_sqrt_f64,
// an LDS write + read round trip, and a 32-bit mad_u64_u32 + xor (Philox).
//   hipcc --offload-arch=gfx950 -O3 -o valu_lat valu_lat.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define N_IT 512

template <int OP>
__global__ void k_lat(unsigned long long* out, double* sink, uint32_t seed) {
  __shared__ double lds[256];
  double f = 1.0 + 1e-9 * threadIdx.x;
  uint32_t a = seed + threadIdx.x;
  lds[threadIdx.x] = f;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
  for (int it = 0; it < N_IT; ++it) {
    if (OP == 0) {
      f = f + 1e-12;
    } else if (OP == 1) {
      f = __fma_rn(f, 0.999999, 1e-7);
    } else if (OP == 2) {
      f = f * 1.0000001;
    } else if (OP == 3) {
      const double g = __builtin_amdgcn_update_dpp(f, f, 0xB1, 0xF, 0xF, true);
      f = f + g * 1e-3;  // dpp move, mul, add
    } else if (OP == 4) {
      f = 1.0 / f + 0.5;
    } else if (OP == 5) {
      f = __builtin_amdgcn_rcp(f) + 0.5;
    } else if (OP == 6) {
      f = __builtin_amdgcn_sqrt(f) + 0.5;
    } else if (OP == 7) {
      lds[threadIdx.x] = f;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      f = lds[threadIdx.x ^ 1] + 1e-12;
    } else if (OP == 8) {
      const uint64_t p = (uint64_t)0xD2511F53u * a;
      a = (uint32_t)(p >> 32) ^ (uint32_t)p ^ 0x9E3779B9u;
    } else if (OP == 9) {
      f = sqrt(f) + 0.5;  // IEEE sqrt sequence
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  sink[blockIdx.x * blockDim.x + threadIdx.x] = f + a;
  if ((threadIdx.x & 63) == 0) out[threadIdx.x / 64] = t1 - t0;
}

template <int OP>
static void run(const char* name, unsigned long long* d_out, double* sink) {
  hipLaunchKernelGGL(k_lat<OP>, dim3(1), dim3(256), 0, 0, d_out, sink, 1u);
  (void)hipDeviceSynchronize();
  unsigned long long h[4];
  (void)hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost);
  unsigned long long mx = 0;
  for (int w = 0; w < 4; ++w) mx = h[w] > mx ? h[w] : mx;
  std::printf("  \"%s\": %.2f,\n", name, (double)mx / N_IT);
}

int main() {
  unsigned long long* d_out;
  double* sink;
  (void)hipMalloc(&d_out, 64 * sizeof(unsigned long long));
  (void)hipMalloc(&sink, 4096 * sizeof(double));
  for (int rep = 0; rep < 2; ++rep) {  // the first pass warms the code
    std::printf("{\"note\": \"dependent-chain cycles per op (s_memtime), one wave per SIMD\",\n");
    run<0>("add_f64", d_out, sink);
    run<1>("fma_f64", d_out, sink);
    run<2>("mul_f64", d_out, sink);
    run<3>("dpp_mul_add_f64", d_out, sink);
    run<4>("ieee_div_f64_plus_add", d_out, sink);
    run<5>("rcp_f64_plus_add", d_out, sink);
    run<6>("hw_sqrt_f64_plus_add", d_out, sink);
    run<7>("lds_write_read_plus_add", d_out, sink);
    run<8>("mad_u64_u32_xor", d_out, sink);
    run<9>("ieee_sqrt_f64_plus_add", d_out, sink);
    std::printf("  \"end\": 0}\n");
  }
  return 0;
}
