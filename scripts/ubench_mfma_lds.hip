// Micro-benchmark: bf16 32x32x16 MFMA chains whose B operand is read from LDS (one ds_read_b128
// per MFMA) while A stays in VGPRs — the inner loop of the register-weight MLP kernel
// (flink_jpmml_amd/ops/csrc/mlp.hip). Reports cycles per MFMA per SIMD for several schedules.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/ubench_mfma_lds.hip -o /tmp/ubench && /tmp/ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int KS = 16;

template <int CH, int W, bool PRIO>
__global__ __launch_bounds__(512, 1) void kern(const uint4* gA, float* out, int iters, unsigned long long* ticks) {
  __shared__ uint4 lds[4 * KS * 64];  // 4 column blocks x 16 k-steps x 64 lanes (64 KiB)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < 4 * KS * 64; i += 512) lds[i] = gA[i & 1023];
  bf16x8 A[KS];
  for (int s = 0; s < KS; ++s) {
    uint4 u = gA[(w * KS + s) * 64 + lane];
    __builtin_memcpy(&A[s], &u, 16);
  }
  __syncthreads();
  f32x16 acc[CH];
  for (int c = 0; c < CH; ++c)
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    const uint4* b[CH];
    for (int c = 0; c < CH; ++c) b[c] = lds + ((c + it) & 3) * KS * 64 + lane;
    uint4 win[CH][W];
#pragma unroll
    for (int i = 0; i < W; ++i)
#pragma unroll
      for (int c = 0; c < CH; ++c) win[c][i] = b[c][i * 64];
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      uint4 x[CH];
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        x[c] = win[c][s % W];
        if (s + W < KS) win[c][s % W] = b[c][(s + W) * 64];
      }
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        bf16x8 B;
        __builtin_memcpy(&B, &x[c], 16);
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[s], B, acc[c], 0, 0, 0);
      }
    }
    if (PRIO) __builtin_amdgcn_s_setprio(0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int c = 0; c < CH; ++c)
    for (int r = 0; r < 16; ++r) s += acc[c][r];
  out[blockIdx.x * 512 + tid] = s;
  if (tid == 0 && blockIdx.x == 0) *ticks = t1 - t0;
}

template <int CH, int W, bool PRIO>
void run(const char* name, const uint4* dA, float* dout, unsigned long long* dt, int ncu) {
  const int iters = 2000;
  hipLaunchKernelGGL((kern<CH, W, PRIO>), dim3(ncu), dim3(512), 0, 0, dA, dout, 10, dt);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((kern<CH, W, PRIO>), dim3(ncu), dim3(512), 0, 0, dA, dout, iters, dt);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long t = 0;
  hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
  const double mfma_per_simd = 2.0 * iters * KS * CH;  // 2 waves per SIMD
  const double flops = 2.0 * 32 * 32 * 16 * (double)iters * KS * CH * 8 * ncu;
  printf("%-28s ticks/MFMA/SIMD %6.1f  %7.1f TFLOP/s  (%.3f ms)\n", name, t / mfma_per_simd, flops / ms / 1e9, ms);
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  std::vector<uint16_t> h(8 * KS * 64 * 8, 0x3c00);
  uint4* dA;
  float* dout;
  unsigned long long* dt;
  hipMalloc(&dA, h.size() * 2);
  hipMemcpy(dA, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  hipMalloc(&dout, ncu * 512 * 4);
  hipMalloc(&dt, 8);
  run<1, 2, false>("1 chain, read-ahead 2", dA, dout, dt, ncu);
  run<1, 4, false>("1 chain, read-ahead 4", dA, dout, dt, ncu);
  run<2, 2, false>("2 chains, read-ahead 2", dA, dout, dt, ncu);
  run<2, 4, false>("2 chains, read-ahead 4", dA, dout, dt, ncu);
  run<2, 2, true>("2 chains, ra 2, setprio", dA, dout, dt, ncu);
  run<4, 1, false>("4 chains, read-ahead 1", dA, dout, dt, ncu);
  run<4, 2, false>("4 chains, read-ahead 2", dA, dout, dt, ncu);
  return 0;
}
