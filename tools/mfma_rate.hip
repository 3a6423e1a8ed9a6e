// Microbenchmark: sustained issue rate of the f32-input MFMA shapes on gfx950 (and bf16 / VALU
// FMA for reference). Each wave runs ITERS x 64 MFMAs over NACC independent accumulators.
// Usage: ./mfma_rate   -> prints TFLOP/s per variant and the in-kernel clock (s_memtime /
// s_memrealtime x 100 MHz).
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef short s8 __attribute__((ext_vector_type(8)));

#define CHECK(x)                                                             \
  do {                                                                       \
    hipError_t e = (x);                                                      \
    if (e != hipSuccess) {                                                   \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);        \
      return 1;                                                              \
    }                                                                        \
  } while (0)

template <int NACC>
__global__ void k16x16x4(float* out, int iters, unsigned long long* clk) {
  f4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f4{0, 0, 0, (float)i};
  float a = threadIdx.x * 1e-3f, b = 1.0f + blockIdx.x * 1e-6f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 64 / NACC; ++j)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int NACC>
__global__ void k32x32x2(float* out, int iters, unsigned long long* clk) {
  f16v acc[NACC];
  for (int i = 0; i < NACC; ++i) for (int j = 0; j < 16; ++j) acc[i][j] = (float)(i + j);
  float a = threadIdx.x * 1e-3f, b = 1.0f + blockIdx.x * 1e-6f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 32 / NACC; ++j)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for (int i = 0; i < NACC; ++i) for (int j = 0; j < 16; ++j) s += acc[i][j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

__global__ void kvalu(float* out, int iters, unsigned long long* clk) {
  float x[16];
  for (int i = 0; i < 16; ++i) x[i] = threadIdx.x * 1e-3f + i;
  float a = 0.999f + blockIdx.x * 1e-9f, b = 1e-3f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) x[i] = fmaf(x[i], a, b);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for (int i = 0; i < 16; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}


// The layer kernel's pattern: A fragments from LDS (ds_read_b128, one step ahead), B operands from a
// 16-register ECL activation, 4 accumulator chains; optional SiLU VALU work on another ECL vector.
template <int MODE>   // 0: frags in registers, 1: frags from LDS each step, 2: + SiLU work
__global__ __launch_bounds__(512) void kpattern(float* out, int iters, unsigned long long* clk) {
  __shared__ __attribute__((aligned(16))) float sW[8192];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 8192; i += blockDim.x) sW[i] = (i % 97) * 1e-3f;
  __syncthreads();
  f4 in[4], acc[4], other[4];
  for (int m = 0; m < 4; ++m) {
    in[m] = f4{lane * 1e-3f, 1.f, 2.f, (float)m};
    acc[m] = f4{0, 0, 0, 0};
    other[m] = f4{0.1f * m, 0.2f, -0.3f, lane * 1e-2f};
  }
  f4 a[4][4];
  for (int mt = 0; mt < 4; ++mt)
    for (int mo = 0; mo < 4; ++mo) a[mt][mo] = *reinterpret_cast<const f4*>(sW + ((mo * 4 + mt) * 64 + lane) * 4);
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
    const float* wf = sW + (it & 1) * 4096;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f4 fr[4];
#pragma unroll
      for (int mo = 0; mo < 4; ++mo)
        fr[mo] = (MODE >= 1) ? *reinterpret_cast<const f4*>(wf + ((mo * 4 + mt) * 64 + lane) * 4) : a[mt][mo];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int mo = 0; mo < 4; ++mo) acc[mo] = __builtin_amdgcn_mfma_f32_16x16x4f32(fr[mo][q], in[mt][q], acc[mo], 0, 0, 0);
      if (MODE == 2) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float x = other[mt][q];
          other[mt][q] = x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)) + 0.5f;
        }
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for (int m = 0; m < 4; ++m) s += acc[m][0] + acc[m][1] + acc[m][2] + acc[m][3] + other[m][0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}


typedef _Float16 h8 __attribute__((ext_vector_type(8)));
// fp16 MFMA 16x16x32 chains (4 accumulators) with optional SiLU VALU work between them.
template <int MODE>   // 0: MFMA only, 1: + 16 SiLU per 16 MFMA (same VALU density per FLOP x 16)
__global__ __launch_bounds__(512) void kf16(float* out, int iters, unsigned long long* clk) {
  const int lane = threadIdx.x & 63;
  h8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)(lane * 1e-3f + j); b[j] = (_Float16)(1.0f - j * 0.01f); }
  f4 acc[4], other[4];
  for (int m = 0; m < 4; ++m) { acc[m] = f4{0, 0, 0, 0}; other[m] = f4{0.1f * m, 0.2f, -0.3f, lane * 1e-2f}; }
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int mo = 0; mo < 4; ++mo) acc[mo] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[mo], 0, 0, 0);
      if (MODE >= 1) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float x = other[mt][q];
          other[mt][q] = x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)) + 0.5f;
        }
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for (int m = 0; m < 4; ++m) s += acc[m][0] + acc[m][1] + acc[m][2] + acc[m][3] + other[m][0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
// fp16 MFMA 16x16x16 (the K = 16 form the edge backward's weight gradients use), 4 accumulators
__global__ __launch_bounds__(512) void kf16k16(float* out, int iters, unsigned long long* clk) {
  const int lane = threadIdx.x & 63;
  h4 a, b;
  for (int j = 0; j < 4; ++j) { a[j] = (_Float16)(lane * 1e-3f + j); b[j] = (_Float16)(1.0f - j * 0.01f); }
  f4 acc[4];
  for (int m = 0; m < 4; ++m) acc[m] = f4{0, 0, 0, 0};
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 16; ++j)
#pragma unroll
      for (int mo = 0; mo < 4; ++mo) acc[mo] = __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, acc[mo], 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for (int m = 0; m < 4; ++m) s += acc[m][0] + acc[m][1] + acc[m][2] + acc[m][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}
// SiLU VALU work alone (same count as the MODE 1/2 variants) to price it
__global__ __launch_bounds__(512) void ksilu(float* out, int iters, unsigned long long* clk) {
  const int lane = threadIdx.x & 63;
  f4 other[4];
  for (int m = 0; m < 4; ++m) other[m] = f4{0.1f * m, 0.2f, -0.3f, lane * 1e-2f};
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float x = other[mt][q];
        other[mt][q] = x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)) + 0.5f;
      }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = other[0][0] + other[3][3];
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <typename K>
int run(const char* name, K kern, int waves_per_block, int blocks, int iters, double flop_per_iter_wave) {
  float* out;
  unsigned long long* clk;
  CHECK(hipMalloc(&out, (size_t)blocks * waves_per_block * 64 * 4));
  CHECK(hipMalloc(&clk, 16));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * waves_per_block), 0, 0, out, iters, clk);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * waves_per_block), 0, 0, out, iters, clk);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long c[2];
  CHECK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  const double flop = flop_per_iter_wave * iters * waves_per_block * blocks;
  printf("%-28s waves/SIMD=%d  %8.3f ms  %7.1f TFLOP/s  clock %.2f GHz\n", name, waves_per_block * blocks / 1024,
         ms, flop / (ms * 1e-3) / 1e12, (double)c[0] / (double)c[1] * 0.1);
  CHECK(hipFree(out));
  CHECK(hipFree(clk));
  return 0;
}

int main() {
  const int iters = 2000;
  for (int wps = 1; wps <= 2; ++wps) {
    const int blocks = 256, wpb = 4 * wps;   // one block per CU, wps waves per SIMD
    run("16x16x4f32 nacc=4", k16x16x4<4>, wpb, blocks, iters, 64.0 * 2048);
    run("16x16x4f32 nacc=8", k16x16x4<8>, wpb, blocks, iters, 64.0 * 2048);
    run("32x32x2f32 nacc=2", k32x32x2<2>, wpb, blocks, iters, 32.0 * 4096);
    run("32x32x2f32 nacc=4", k32x32x2<4>, wpb, blocks, iters, 32.0 * 4096);
    run("valu fma x16", kvalu, wpb, blocks, iters, 8.0 * 16 * 64 * 2);
    run("pattern regs", kpattern<0>, wpb, blocks, iters, 64.0 * 2048);
    run("pattern lds-frags", kpattern<1>, wpb, blocks, iters, 64.0 * 2048);
    run("pattern lds-frags+silu", kpattern<2>, wpb, blocks, iters, 64.0 * 2048);
    run("f16 16x16x32 x64", kf16<0>, wpb, blocks, iters, 64.0 * 16384);
    run("f16 16x16x32 x64 + 16 silu", kf16<1>, wpb, blocks, iters, 64.0 * 16384);
    run("16 silu alone (flop=f16 eq)", ksilu, wpb, blocks, iters, 64.0 * 16384);
    run("f16 16x16x16 x64", kf16k16, wpb, blocks, iters, 64.0 * 8192);
  }
  return 0;
}
